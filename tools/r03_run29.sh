set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/t29.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/t29.log; exit 1; }
tail -2 gpurun_out/r03/t29.log
timeout -k 10 600 bash tools/ab.sh gpurun_out/r03/ab29 merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 -- ab/libbsg_head.so ab/libbsg_laload.so ab/libbsg_laprio.so > gpurun_out/r03/ab29.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03/ab29.txt; exit 1; }
cat gpurun_out/r03/ab29.txt
