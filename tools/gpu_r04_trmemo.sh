#!/bin/bash
# Turn-rate memo (keyed by tas): the whole GPU suite, then A/B (tools/_var: base = HEAD,
# trmemo).  GPU box, repo root.
set -uo pipefail
OUT=gpurun_out/${1:-r04trmemo}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo tests failed; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -n 1 "$OUT/gpu_tests.log"
ABL="merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048" bash tools/ab.sh "$OUT/ab" merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 -- tools/_var/libbsg_base.so tools/_var/libbsg_trmemo.so > "$OUT/ab.txt" 2>&1 || exit 1
cat "$OUT/ab.txt"
