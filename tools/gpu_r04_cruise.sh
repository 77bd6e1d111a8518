#!/bin/bash
# The cruise substep of the lookahead waves: bit-identity tests, then A/B against HEAD's kernel.
set -uo pipefail
OUT=gpurun_out/${1:-r04cruise}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
bash tools/ab.sh "$OUT/ab" merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 -- tools/_var/libbsg_head.so tools/_var/libbsg_cruise.so > "$OUT/ab.txt" 2>&1 || exit 1
