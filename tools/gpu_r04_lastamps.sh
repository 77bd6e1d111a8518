#!/bin/bash
# Lookahead-wave stamps (resetting vs not) of the C4 shards.  GPU box, repo root.
set -uo pipefail
OUT=gpurun_out/${1:-r04lastamps}
mkdir -p "$OUT"
for E in 512 1024; do
  BSG_LIBRARY=$PWD/tools/_var/libbsg_stamps.so timeout -k 10 240 python3 -u tools/stamps.py $E 32 > "$OUT/stamps_$E.txt" 2>&1 || { echo "stamps $E failed"; tail -20 "$OUT/stamps_$E.txt"; exit 1; }
done
tail -12 "$OUT/stamps_512.txt"
