#!/bin/bash
# One GPU-box validation pass: pytest -m gpu, smoke(), bench, rocprofv3 stats + PMC.
# Usage (on the box, from the repo root):  bash tools/gpu_round.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-r02}
KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" ; date +%T
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
if [ -n "$KEXPR" ]; then
  run gpu_tests 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "$KEXPR" || exit 1
else
  run gpu_tests 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread || exit 1
fi
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 600 python bench.py || exit 1
grep "^{" "$OUT/bench.log" > "$OUT/bench.json"
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
run profile 900 bash tools/profile.sh "$TAG" || exit 1
