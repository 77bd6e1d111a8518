#!/bin/bash
# rocprofv3 kernel-trace summary of BASELINE configs[4] (bench.py --workload descent-sac:
# DescentEnv-v0 x 4096 with the SAC learner in the loop), per kernel, for the learner's
# launch breakdown.  Run on the GPU box from the repo root:  bash tools/profile_c5.sh r05
set -euo pipefail
TAG=${1:-r05}
STEPS=${STEPS:-200}
OUT=gpurun_out/prof_c5_$TAG
mkdir -p "$OUT" "profiles/$TAG"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --workload descent-sac --steps "$STEPS" --warmup 20 > "$OUT/bench.json"
f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
cp "$f" "profiles/$TAG/c5_kernel_stats.csv"
cp "$OUT/bench.json" "profiles/$TAG/c5_bench.json"
