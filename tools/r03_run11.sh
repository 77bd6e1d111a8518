set -o pipefail
mkdir -p gpurun_out/r03
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
timeout -k 10 150 python tools/probe/substep_probe.py tools/probe/substep_probe_base tools/probe/substep_probe > gpurun_out/r03/probe_aadd.txt 2>&1 || { echo PROBE_FAILED; tail gpurun_out/r03/probe_aadd.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/probe_aadd.txt | grep -v "substep [0-9]*:"
timeout -k 10 900 bash tools/ab.sh gpurun_out/r03/ab_x merge32_full merge32_full_512 vert32_full_2048 descent_4096 -- $L/libbsg_base.so $L/libbsg.so $L/libbsg_x1.so $L/libbsg_x2.so $L/libbsg_x3.so > gpurun_out/r03/ab_x.txt 2>&1 || { echo AB_FAILED; tail gpurun_out/r03/ab_x.txt; exit 1; }
cat gpurun_out/r03/ab_x.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/gpu_aadd.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/gpu_aadd.log; exit 1; }
tail -2 gpurun_out/r03/gpu_aadd.log
