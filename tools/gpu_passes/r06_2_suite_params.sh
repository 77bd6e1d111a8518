#!/bin/bash
# Round-6 GPU pass 2: the whole GPU suite on the build with the Merge constants as kernel
# parameters, then the default bench line.
set -uo pipefail
OUT=gpurun_out/r06b
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 4 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
step gpu_tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step bench 300 python -u bench.py --steps 200 --warmup 20 || exit 1
