set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 bash tools/ab.sh gpurun_out/r03/ab36 vert32_full_2048 vert32_full_1024 -- ab/libbsg_cur.so ab/libbsg_vprio0.so > gpurun_out/r03/ab36.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03/ab36.txt; exit 1; }
cat gpurun_out/r03/ab36.txt
