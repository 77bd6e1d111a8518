#!/bin/bash
# The RCCL transport after the fused step+gather call: tests, the overhead table, the
# per-part host breakdown (BSG_COMM_PROFILE=1).
set -uo pipefail
OUT=gpurun_out/${1:-r04e}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread -k rccl > "$OUT/sharded.log" 2>&1 || exit 1
BSG_COMM_PROFILE=1 timeout -k 10 300 python -u tools/shard_overhead_nccl.py > "$OUT/shard_overhead.txt" 2>&1 || exit 1
for g in 0 1; do
  BSG_COMM_GRAPHS=$g BSG_COMM_PROFILE=1 timeout -k 10 120 python -u tools/shard_host_breakdown.py 512 1 rccl > "$OUT/host_rccl_g$g.txt" 2>&1 || exit 1
done
