#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the
# bench workload.  Run on the GPU box from the repo root:  bash tools/profile.sh r01
set -euo pipefail
TAG=${1:-r01}
STEPS=${STEPS:-50}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps "$STEPS" --warmup 5 --skip-cpu-baseline > "$OUT/bench_trace.json"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 bench.py --steps "$STEPS" --warmup 5 --skip-cpu-baseline > "$OUT/bench_fetch.json"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 bench.py --steps "$STEPS" --warmup 5 --skip-cpu-baseline > "$OUT/bench_write.json"
find "$OUT" -name "*.csv" | sort > "$OUT/files.txt"
