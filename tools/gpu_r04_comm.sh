#!/bin/bash
# Round-4 multi-GPU path on one box: the RCCL-transport tests, the host-overhead table
# (torch all_gather vs libbsg bsg_comm, graph-replayed and plain), the default bench line
# (with C5's learner leg) and a 2-rank gloo rehearsal of `bench.py --gpus 2`.
set -uo pipefail
OUT=gpurun_out/${1:-r04c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread > "$OUT/sharded.log" 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_overhead_nccl.py > "$OUT/shard_overhead.txt" 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || exit 1
BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29577 bench.py --gpus 2 --steps 20 --warmup 5 > "$OUT/bench_2rank_gloo.log" 2>&1 || exit 1
