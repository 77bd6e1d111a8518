set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_fastpath.py tests/test_gpu_lookahead.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03/fast27_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/fast27_tests.log; exit 1; }
tail -3 gpurun_out/r03/fast27_tests.log
CF="merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048"
for rep in 1 2; do
for v in "def:" "old:BSG_NO_FASTPATH=1"; do
  n=${v%%:*}; envs=${v#*:}
  env $envs ABLATE_OUT=gpurun_out/r03/ab27_${n}_$rep.json timeout -k 10 200 python -u tools/ablate.py $CF > gpurun_out/r03/ab27_${n}_$rep.txt 2>&1 || { echo ABLATE_FAILED $n; tail -20 gpurun_out/r03/ab27_${n}_$rep.txt; exit 1; }
done
done
for f in gpurun_out/r03/ab27_*.txt; do echo "== $f"; grep us $f; done
export BSG_LIBRARY=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg_stamps.so
for E in 512 2048; do
  timeout -k 10 240 python -u tools/stamps.py $E 32 > gpurun_out/r03/st27_$E.txt 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/r03/st27_$E.txt; exit 1; }
  sed -n 2,13p gpurun_out/r03/st27_$E.txt; grep -A6 "lookahead waves" gpurun_out/r03/st27_$E.txt
done
