#!/bin/bash
# Round-6 GPU pass 3: the trajectory store -- its bit-identity tests, the lookahead / parity /
# sharded suites it now runs under, then the C4 shard timings with it on and off.
set -uo pipefail
OUT=gpurun_out/r06c
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 6 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
step tj_tests 600 python -u -m pytest tests/test_gpu_trajectory.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step la_tests 900 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step sweep_tj 300 python -u tools/shard_gather_sweep.py 512 1024 2048 || exit 1
BSG_TRAJECTORY=0 step sweep_notj 300 python -u tools/shard_gather_sweep.py 512 1024 || exit 1
L=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib
for e in 512 1024; do
  BSG_LIBRARY=$L/libbsg_stamps.so step stamps_$e 120 python -u tools/stamps.py $e 32 || exit 1
done
