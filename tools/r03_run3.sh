set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_fastpath.py tests/test_gpu_lookahead.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_fast.log 2>&1 || { echo FAST_FAILED; tail -30 gpurun_out/r03/gpu_fast.log; exit 1; }
tail -2 gpurun_out/r03/gpu_fast.log
timeout -k 10 200 python tools/ablate.py merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 vert32_full_2048 descent_4096 descent_512 > gpurun_out/r03/ablate_c.txt 2>&1; grep -v amdgpu.ids gpurun_out/r03/ablate_c.txt
timeout -k 10 300 python bench.py > gpurun_out/r03/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03/bench.log; exit 1; }
grep "^{" gpurun_out/r03/bench.log > gpurun_out/r03/bench.json
timeout -k 10 900 bash tools/profile.sh r03 > gpurun_out/r03/profile.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r03/profile.log; exit 1; }
tail -3 gpurun_out/r03/profile.log
timeout -k 10 600 bash tools/ab.sh gpurun_out/r03/ab_w4 merge32_full merge32_full_la merge32_full_512 -- bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg.so bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg_w4.so > gpurun_out/r03/ab_w4.txt 2>&1; cat gpurun_out/r03/ab_w4.txt
