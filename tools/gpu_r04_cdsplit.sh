#!/bin/bash
# CD phase 2, one pair order per lane: per-wave stamps of the C4 shards (HEAD build), the CD
# parity / bit-identity tests on the new build, then A/B (tools/_var: base = HEAD, cdsplit).
set -uo pipefail
OUT=gpurun_out/${1:-r04cdsplit}
mkdir -p "$OUT"
export TMPDIR=/tmp
for E in 512 1024; do
  BSG_LIBRARY=$PWD/tools/_var/libbsg_stamps.so timeout -k 10 240 python3 -u tools/stamps.py $E 32 > "$OUT/stamps_$E.txt" 2>&1 || { echo "stamps $E failed"; exit 1; }
done
echo stamps done
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py tests/test_gpu_areas.py tests/test_gpu_plan.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo tests failed; tail -30 "$OUT/tests.log"; exit 1; }
echo tests done
bash tools/ab.sh "$OUT/ab" merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 -- tools/_var/libbsg_base.so tools/_var/libbsg_cdsplit.so > "$OUT/ab.txt" 2>&1 || exit 1
cat "$OUT/ab.txt"
