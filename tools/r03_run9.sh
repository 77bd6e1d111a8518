set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 120 tools/probe/atan2_probe > gpurun_out/r03/atan2_probe.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03/atan2_probe.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 120 tools/probe/fastmath_probe > gpurun_out/r03/fastmath_probe.txt 2>&1 || { echo FM_FAILED; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/fastmath_probe.txt | head -20
timeout -k 10 150 python tools/probe/substep_probe.py tools/probe/substep_probe_base tools/probe/substep_probe > gpurun_out/r03/probe_fmak.txt 2>&1 || { echo PROBE_FAILED; tail gpurun_out/r03/probe_fmak.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/probe_fmak.txt | grep -v "substep [0-9]*:"
timeout -k 10 600 bash tools/ab.sh gpurun_out/r03/ab_fmak merge32_full merge32_full_512 vert32_full_2048 descent_4096 -- bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg_base.so bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg.so > gpurun_out/r03/ab_fmak.txt 2>&1 || { echo AB_FAILED; tail gpurun_out/r03/ab_fmak.txt; exit 1; }
cat gpurun_out/r03/ab_fmak.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/gpu_fmak.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/gpu_fmak.log; exit 1; }
tail -2 gpurun_out/r03/gpu_fmak.log
