#!/bin/bash
# Round-6 GPU pass 8: the trajectory store's producer throttles at 512 / 1024 envs.
set -uo pipefail
OUT=gpurun_out/r06h
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 2 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
step tj_tests 600 python -u -m pytest tests/test_gpu_trajectory.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
for E in 512 1024; do
  step off_$E 120 python -u tools/traj_ab.py --mode off $E || exit 1
  step on_$E 120 python -u tools/traj_ab.py --mode on $E || exit 1
  BSG_TRAJ_EVERY=8 step every8_$E 120 python -u tools/traj_ab.py --mode on $E || exit 1
  BSG_TRAJ_EVERY=8 BSG_TRAJ_SLEEP=6 step every8_sleep6_$E 120 python -u tools/traj_ab.py --mode on $E || exit 1
  BSG_TRAJ_EVERY=4 BSG_TRAJ_SLEEP=12 step every4_sleep12_$E 120 python -u tools/traj_ab.py --mode on $E || exit 1
done
