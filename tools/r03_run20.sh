set -o pipefail
mkdir -p gpurun_out/r03
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
timeout -k 10 900 bash tools/ab.sh gpurun_out/r03/ab_abl merge32_full merge32_full_512 -- $L/libbsg.so $L/libbsg_a1.so $L/libbsg_a2.so $L/libbsg_a3.so $L/libbsg_a4.so $L/libbsg_a5.so > gpurun_out/r03/ab_abl.txt 2>&1 || { echo AB_FAILED; tail gpurun_out/r03/ab_abl.txt; exit 1; }
cat gpurun_out/r03/ab_abl.txt
