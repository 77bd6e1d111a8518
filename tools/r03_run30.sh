set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/t30.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03/t30.log; exit 1; }
tail -2 gpurun_out/r03/t30.log
for rep in 1 2; do
timeout -k 10 300 python -u tools/ablate.py vert32_full_2048 vert32_full_2048_nola vert32_full_1024 vert32_full_1024_nola merge32_full_512 > gpurun_out/r03/ab30_$rep.txt 2>&1 || { echo ABLATE_FAILED; tail -20 gpurun_out/r03/ab30_$rep.txt; exit 1; }
grep us gpurun_out/r03/ab30_$rep.txt
done
