#!/bin/bash
# Merge spawn cache: bit-identity / parity tests, A/B against HEAD (tools/_var: base,
# spawncache), then per-wave stamps of the C4 shards on the new build.  GPU box, repo root.
set -uo pipefail
OUT=gpurun_out/${1:-r04spawncache}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_fastpath.py tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo tests failed; tail -30 "$OUT/tests.log"; exit 1; }
echo tests done
bash tools/ab.sh "$OUT/ab" merge32_full merge32_full_512 merge32_full_1024 merge32_full_2048 -- tools/_var/libbsg_base.so tools/_var/libbsg_spawncache.so > "$OUT/ab.txt" 2>&1 || exit 1
cat "$OUT/ab.txt"
for E in 512 1024; do
  BSG_LIBRARY=$PWD/tools/_var/libbsg_stamps.so timeout -k 10 240 python3 -u tools/stamps.py $E 32 > "$OUT/stamps_$E.txt" 2>&1 || { echo "stamps $E failed"; exit 1; }
done
tail -12 "$OUT/stamps_512.txt"
