#!/bin/bash
# Round-6 GPU pass 4: trajectory store A/B (off / on / on without async producers) and the
# per-wave stamps of a 512-env shard with it on and copy-only.
set -uo pipefail
OUT=gpurun_out/r06d
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
step traj_ab 600 python -u tools/traj_ab.py 512 1024 || exit 1
L=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib
BSG_LIBRARY=$L/libbsg_stamps.so step stamps_512_tj 120 python -u tools/stamps.py 512 32 || exit 1
BSG_TRAJ_NOASYNC=1 BSG_LIBRARY=$L/libbsg_stamps.so step stamps_512_copyonly 120 python -u tools/stamps.py 512 32 || exit 1
BSG_TRAJECTORY=0 BSG_LIBRARY=$L/libbsg_stamps.so step stamps_512_off 120 python -u tools/stamps.py 512 32 || exit 1
