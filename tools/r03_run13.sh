set -o pipefail
mkdir -p gpurun_out/r03
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
timeout -k 10 900 bash tools/ab.sh gpurun_out/r03/ab_h merge32_full merge32_full_512 vert32_full_2048 descent_4096 -- $L/libbsg_base.so $L/libbsg.so $L/libbsg_x4.so > gpurun_out/r03/ab_h.txt 2>&1 || { echo AB_FAILED; tail gpurun_out/r03/ab_h.txt; exit 1; }
cat gpurun_out/r03/ab_h.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/gpu_h.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/gpu_h.log; exit 1; }
tail -2 gpurun_out/r03/gpu_h.log
BSG_LIBRARY=$PWD/$L/libbsg_x4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lookahead.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/gpu_h4.log 2>&1 || { echo TESTS4_FAILED; tail -30 gpurun_out/r03/gpu_h4.log; exit 1; }
tail -2 gpurun_out/r03/gpu_h4.log
timeout -k 10 120 python -u tools/shard_host_breakdown.py 512 > gpurun_out/r03/shard_host_breakdown.txt 2>&1 || { echo BD_FAILED; tail gpurun_out/r03/shard_host_breakdown.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/shard_host_breakdown.txt | grep "E="
