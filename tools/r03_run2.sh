set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python bench.py > gpurun_out/r03/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03/bench.log; exit 1; }
grep "^{" gpurun_out/r03/bench.log > gpurun_out/r03/bench.json
timeout -k 10 900 bash tools/profile.sh r03 > gpurun_out/r03/profile.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r03/profile.log; exit 1; }
tail -5 gpurun_out/r03/profile.log
