#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes for the bench workload.
# Run on the GPU box from the repo root:  bash tools/profile.sh r01
# Writes gpurun_out/prof_<tag>/ and the summaries profiles/<tag>/{kernel_stats.csv,pmc.json}.
set -euo pipefail
TAG=${1:-r01}
STEPS=${STEPS:-50}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT" "profiles/$TAG"
export TMPDIR=/tmp
B="python3 bench.py --steps $STEPS --warmup 5 --skip-cpu-baseline --no-c5"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B > "$OUT/bench_trace.json"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $B > /dev/null
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- $B > /dev/null
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/pmc_valu" -o run -- $B > /dev/null
python3 tools/profile_summary.py "$OUT" "$TAG"
