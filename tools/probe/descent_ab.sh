#!/bin/bash
# Descent 4096 env-only / env+policy / learner legs (bench.py --workload descent-sac) under
# several builds of libbsg (bluesky_gym/_lib/libbsg_<v>.so; "new" = libbsg.so), alternating.
# On the GPU box from the repo root:  bash tools/probe/descent_ab.sh <tag> <v1> <v2> ...
set -euo pipefail
TAG=${1:-descent_ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
for r in 1 2; do
  for v in "$@"; do
    lib=$L/libbsg_$v.so; [ $v = new ] && lib=$L/libbsg.so
    BSG_LIBRARY=$lib timeout -k 10 300 python bench.py --workload descent-sac --steps 300 --warmup 20 2>/dev/null \
      | grep "^{" > "$OUT/${v}_$r.json"
    python -c "import json;d=json.load(open('$OUT/${v}_$r.json'));print('$v', $r, 'env_only', round(d['env_only']['ms_per_step']*1e3,2), 'us  env_policy', round(d['env_policy']['ms_per_step']*1e3,2), 'us  learner', round(d['ms_per_step']*1e3,1), 'us')"
  done
done
