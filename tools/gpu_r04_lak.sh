#!/bin/bash
# Lookahead-free instance for launches without the lookahead (LAK) on top of the cruise
# re-check and the created aircraft's memo keys: the whole GPU suite, then A/B (tools/_var:
# base = HEAD, spawnmemo = re-check + memo keys, lak = + the instance split).
set -uo pipefail
OUT=gpurun_out/${1:-r04lak}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo tests failed; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -n 2 "$OUT/gpu_tests.log"
bash tools/ab.sh "$OUT/ab" merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 -- tools/_var/libbsg_base.so tools/_var/libbsg_spawnmemo.so tools/_var/libbsg_lak.so > "$OUT/ab.txt" 2>&1 || exit 1
cat "$OUT/ab.txt"
