#!/bin/bash
# Round-6 GPU pass 7: device-published producers -- trajectory / lookahead tests, then the A/B.
set -uo pipefail
OUT=gpurun_out/r06g
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 8 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
step tj_tests 600 python -u -m pytest tests/test_gpu_trajectory.py tests/test_gpu_lookahead.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step traj_ab 600 python -u tools/traj_ab.py 512 1024 || exit 1
