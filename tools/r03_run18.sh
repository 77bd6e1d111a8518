set -o pipefail
mkdir -p gpurun_out/r03
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
timeout -k 10 900 bash tools/ab.sh gpurun_out/r03/ab_route vert32_full_2048 merge32_full descent_4096 vert32_full_2048 -- $L/libbsg_base.so $L/libbsg.so > gpurun_out/r03/ab_route.txt 2>&1 || { echo AB_FAILED; tail gpurun_out/r03/ab_route.txt; exit 1; }
cat gpurun_out/r03/ab_route.txt
