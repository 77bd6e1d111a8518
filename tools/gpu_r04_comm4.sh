#!/bin/bash
# The fused per-step gather after the flag / fence / priority change: the sharded and
# lookahead GPU tests, the host-overhead table and the per-part host breakdown.
set -uo pipefail
OUT=gpurun_out/${1:-r04comm4}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_lookahead.py -x -v --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
BSG_COMM_PROFILE=1 timeout -k 10 300 python -u tools/shard_overhead_nccl.py > "$OUT/shard_overhead.txt" 2>&1 || exit 1
BSG_COMM_PROFILE=1 timeout -k 10 120 python -u tools/shard_host_breakdown.py 512 1 rccl > "$OUT/host_rccl.txt" 2>&1 || exit 1
