#!/bin/bash
# C5 learner-in-the-loop rate against RL iterations per HIP graph replay (C5_GRAPH_ITERS)
set -euo pipefail
mkdir -p gpurun_out/c5k
for k in 1 2 4 8; do
  C5_GRAPH_ITERS=$k timeout -k 10 300 python bench.py --workload descent-sac --steps 400 --warmup 24 | grep "^{" > gpurun_out/c5k/k$k.json
  echo "k=$k"; python -c "import json;d=json.load(open('gpurun_out/c5k/k$k.json'));print(d['value'],d['ms_per_step'],d['env_policy'])"
done
