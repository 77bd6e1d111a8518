#!/bin/bash
# Round-6 GPU pass 6: why the producers lag -- their queue / wave priorities A/B, and a
# kernel trace of the store in steady state.
set -uo pipefail
OUT=gpurun_out/r06f
mkdir -p "$OUT"
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
for E in 512 1024; do
  BSG_TRAJ_WPRIO=1 step ab_least_w1_$E 120 python -u tools/traj_ab.py --mode on $E || exit 1
  BSG_TRAJ_WPRIO=0 step ab_least_w0_$E 120 python -u tools/traj_ab.py --mode on $E || exit 1
  BSG_TRAJ_QPRIO=normal BSG_TRAJ_WPRIO=1 step ab_normal_w1_$E 120 python -u tools/traj_ab.py --mode on $E || exit 1
  BSG_TRAJ_QPRIO=normal BSG_TRAJ_WPRIO=0 step ab_normal_w0_$E 120 python -u tools/traj_ab.py --mode on $E || exit 1
done
step trace_512 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace512 -o run -- python3 tools/traj_ab.py --mode on 512 || exit 1
