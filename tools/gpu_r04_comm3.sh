#!/bin/bash
# Round-4 multi-GPU evidence in one call: the sharded tests (k = 1 and blocks, torch and
# native RCCL transports), the host-overhead table, the per-part host breakdown of the fused
# bsg_step_gather call, and 2-rank gloo rehearsals of `bench.py --gpus 2` (default k = 1 line
# with its gather_block variant).
set -uo pipefail
OUT=gpurun_out/${1:-r04comm}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread > "$OUT/sharded.log" 2>&1 || exit 1
BSG_COMM_PROFILE=1 timeout -k 10 300 python -u tools/shard_overhead_nccl.py > "$OUT/shard_overhead.txt" 2>&1 || exit 1
for g in 0 1; do
  BSG_COMM_GRAPHS=$g BSG_COMM_PROFILE=1 timeout -k 10 120 python -u tools/shard_host_breakdown.py 512 1 rccl > "$OUT/host_rccl_g$g.txt" 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/shard_host_breakdown.py 512 1 torch > "$OUT/host_torch.txt" 2>&1 || exit 1
BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29577 bench.py --gpus 2 --steps 20 --warmup 5 --no-c5 > "$OUT/bench_2rank_gloo.log" 2>&1 || exit 1
