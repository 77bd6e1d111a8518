set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookahead.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_la.log 2>&1 || { echo LA_FAILED; tail -30 gpurun_out/r03/gpu_la.log; exit 1; }
tail -2 gpurun_out/r03/gpu_la.log
timeout -k 10 240 python tools/ablate.py merge32_full merge32_full_la merge32_full_512 merge32_full_512_nola merge32_full_1024 merge32_full_1024_nola merge32_full_2048 merge32_full_2048_nola vert32_full_2048 descent_4096 > gpurun_out/r03/ablate_b.txt 2>&1; grep -v amdgpu.ids gpurun_out/r03/ablate_b.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_tests_b.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/gpu_tests_b.log; exit 1; }
tail -2 gpurun_out/r03/gpu_tests_b.log
timeout -k 10 120 python tools/probe/substep_probe.py --descent tools/probe/substep_probe_d > gpurun_out/r03/probe_descent_b.txt 2>&1; tail -3 gpurun_out/r03/probe_descent_b.txt
