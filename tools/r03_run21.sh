set -o pipefail
mkdir -p gpurun_out/r03
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
timeout -k 10 900 bash tools/ab.sh gpurun_out/r03/ab_prio merge32_full merge32_full_2048 -- $L/libbsg.so $L/libbsg_p23.so $L/libbsg_p45.so $L/libbsg_p0.so > gpurun_out/r03/ab_prio.txt 2>&1 || { echo AB_FAILED; tail gpurun_out/r03/ab_prio.txt; exit 1; }
cat gpurun_out/r03/ab_prio.txt
