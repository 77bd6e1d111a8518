#!/bin/bash
# Round-6 final GPU pass: the whole GPU suite, smoke(), the default bench line, the rocprofv3
# kernel-trace summary + PMC passes of the headline (tools/profile.sh r06), the configs'
# kernel stats + PMC (tools/profile_configs.sh r06) and the C4 gather sweep.
set -uo pipefail
TAG=${1:-r06}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" "profiles/$TAG"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
step gpu_tests 1100 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc      # (1: test failures -- keep measuring)
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python bench.py || exit 1
grep "^{" "$OUT/bench.log" > "profiles/$TAG/bench.json"
step profile 900 bash tools/profile.sh "$TAG" || exit 1
step profile_configs 900 bash tools/profile_configs.sh "$TAG" || exit 1
python3 tools/profile_configs_summary.py gpurun_out/profcfg_$TAG "$TAG" > "$OUT/profile_configs_summary.log" 2>&1
step gather_sweep 300 python -u tools/shard_gather_sweep.py 512 1024 2048 4096 || exit 1
# profiles/<tag>/ written on the box travel back under gpurun_out/
mkdir -p "$OUT/profiles_copy" && cp -r "profiles/$TAG/." "$OUT/profiles_copy/" && cp profiles/traffic.json "$OUT/profiles_copy/traffic.json"
