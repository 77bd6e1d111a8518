set -o pipefail
mkdir -p gpurun_out/r03
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
timeout -k 10 900 bash tools/ab.sh gpurun_out/r03/ab_rs merge32_full merge32_full_512 vert32_full_2048 descent_4096 -- $L/libbsg_base.so $L/libbsg.so > gpurun_out/r03/ab_rs.txt 2>&1 || { echo AB_FAILED; tail gpurun_out/r03/ab_rs.txt; exit 1; }
cat gpurun_out/r03/ab_rs.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py tests/test_gpu_plan.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/gpu_rs.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/gpu_rs.log; exit 1; }
tail -2 gpurun_out/r03/gpu_rs.log
