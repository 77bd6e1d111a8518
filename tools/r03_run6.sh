set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_tests_c.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/gpu_tests_c.log; exit 1; }
tail -2 gpurun_out/r03/gpu_tests_c.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03/smoke.log 2>&1 || { echo SMOKE_FAILED; tail gpurun_out/r03/smoke.log; exit 1; }
tail -1 gpurun_out/r03/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r03/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03/bench.log; exit 1; }
grep "^{" gpurun_out/r03/bench.log > gpurun_out/r03/bench.json
