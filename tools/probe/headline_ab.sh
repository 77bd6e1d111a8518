#!/bin/bash
# Headline kernel A/B (MergeEnv 4096 x 32, bench.py's HIP-event kernel average) under two
# builds of libbsg, alternating: bash tools/probe/headline_ab.sh <tag> <v1> <v2> ...
# ("new" = libbsg.so, otherwise bluesky_gym/_lib/libbsg_<v>.so)
set -euo pipefail
TAG=${1:-headline_ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
for r in 1 2 3; do
  for v in "$@"; do
    lib=$L/libbsg_$v.so; [ $v = new ] && lib=$L/libbsg.so
    BSG_LIBRARY=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 20 --skip-cpu-baseline --no-c5 2>/dev/null \
      | grep "^{" > "$OUT/${v}_$r.json"
    python -c "import json;d=json.load(open('$OUT/${v}_$r.json'));print('$v', $r, 'kernel', round(d['roofline']['kernel_avg_ms']*1e3,2), 'us  wall', round(d['ms_per_step']*1e3,2), 'us')"
  done
done
