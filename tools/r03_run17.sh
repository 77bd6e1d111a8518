set -o pipefail
mkdir -p gpurun_out/r03
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
timeout -k 10 900 bash tools/ab.sh gpurun_out/r03/ab_cd2 merge32_full merge32_full_512 vert32_full_2048 -- $L/libbsg_base.so $L/libbsg_p0.so $L/libbsg.so > gpurun_out/r03/ab_cd2.txt 2>&1 || { echo AB_FAILED; tail gpurun_out/r03/ab_cd2.txt; exit 1; }
cat gpurun_out/r03/ab_cd2.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lookahead.py tests/test_gpu_areas.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/gpu_cd2.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/gpu_cd2.log; exit 1; }
tail -2 gpurun_out/r03/gpu_cd2.log
