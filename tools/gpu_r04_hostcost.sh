#!/bin/bash
# Host cost of one sharded step, torch vs libbsg's RCCL transport (plain and graph-replayed
# gathers), with the C call's own breakdown (BSG_COMM_PROFILE=1).
set -uo pipefail
OUT=gpurun_out/${1:-r04d}
mkdir -p "$OUT"
for tr in torch rccl; do
  for g in 0 1; do
    BSG_COMM_GRAPHS=$g BSG_COMM_PROFILE=1 timeout -k 10 120 python -u tools/shard_host_breakdown.py 512 1 $tr \
      > "$OUT/host_${tr}_g$g.txt" 2>&1 || exit 1
    [ $tr = torch ] && break
  done
done
