#!/bin/bash
# Cruise re-check after each general substep + a created aircraft's memo keys: bit-identity
# tests, A/B (tools/_var: base = HEAD, recheck, spawnmemo = both), stamps.  GPU box, repo root.
set -uo pipefail
OUT=gpurun_out/${1:-r04recheck}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo tests failed; tail -30 "$OUT/tests.log"; exit 1; }
echo tests done
bash tools/ab.sh "$OUT/ab" merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 -- tools/_var/libbsg_base.so tools/_var/libbsg_recheck.so tools/_var/libbsg_spawnmemo.so > "$OUT/ab.txt" 2>&1 || exit 1
cat "$OUT/ab.txt"
BSG_LIBRARY=$PWD/tools/_var/libbsg_stamps.so timeout -k 10 240 python3 -u tools/stamps.py 512 32 > "$OUT/stamps_512.txt" 2>&1 || { echo "stamps failed"; exit 1; }
tail -14 "$OUT/stamps_512.txt"
