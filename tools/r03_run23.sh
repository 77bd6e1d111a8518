set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/gpu_shard2.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/gpu_shard2.log; exit 1; }
tail -2 gpurun_out/r03/gpu_shard2.log
SKIP_PROF=1 bash tools/gpu_round.sh r03c || { echo ROUND_FAILED; exit 1; }
