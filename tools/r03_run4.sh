set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_fastpath.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_fast2.log 2>&1 || { echo FAST_FAILED; tail -30 gpurun_out/r03/gpu_fast2.log; exit 1; }
tail -2 gpurun_out/r03/gpu_fast2.log
timeout -k 10 120 python tools/probe/substep_probe.py --descent tools/probe/fast_probe tools/probe/substep_probe_d > gpurun_out/r03/probe_fast.txt 2>&1; grep -v amdgpu.ids gpurun_out/r03/probe_fast.txt | grep -v "substep [0-9]*:"
timeout -k 10 200 python tools/ablate.py vert32_full_2048 descent_4096 descent_512 > gpurun_out/r03/ablate_d.txt 2>&1; grep -v amdgpu.ids gpurun_out/r03/ablate_d.txt
