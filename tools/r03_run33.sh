set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/t33.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03/t33.log; exit 1; }
tail -2 gpurun_out/r03/t33.log
timeout -k 10 600 bash tools/ab.sh gpurun_out/r03/ab33 vert32_full_2048 vert32_full_1024 merge32_full merge32_full_512 -- ab/libbsg_head2.so ab/libbsg_vlacd.so > gpurun_out/r03/ab33.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03/ab33.txt; exit 1; }
cat gpurun_out/r03/ab33.txt
