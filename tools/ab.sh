#!/bin/bash
# A/B kernel timing on one GPU box: alternate ablate.py runs over the libraries given
# (BSG_LIBRARY), so box-to-box variance cancels.  Usage: bash tools/ab.sh OUTDIR cfgs -- lib...
set -uo pipefail
OUT=$1; shift
CFGS=()
while [ "$1" != "--" ]; do CFGS+=("$1"); shift; done
shift
mkdir -p "$OUT"
for round in 1 2; do
  for lib in "$@"; do
    echo "== $(basename $lib) round $round"
    BSG_LIBRARY=$PWD/$lib ABLATE_OUT=$OUT/$(basename $lib .so)_$round.json \
      timeout -k 10 200 python tools/ablate.py "${CFGS[@]}" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
