#!/bin/bash
# Merge spawn constants + memo prefill: bit-identity / parity tests, then A/B against the
# previous kernel (tools/_var: cruise = before, spawnk = after).
set -uo pipefail
OUT=gpurun_out/${1:-r04spawnk}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
bash tools/ab.sh "$OUT/ab" merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 -- tools/_var/libbsg_cruise.so tools/_var/libbsg_spawnk.so > "$OUT/ab.txt" 2>&1 || exit 1
