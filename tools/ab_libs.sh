#!/bin/bash
# Round-robin A/B of several libbsg builds on one box (tools/ab_tree.py timing):
#   bash tools/ab_libs.sh "<lib> <lib> ..." rounds E...
set -uo pipefail
LIBS=$1; R=$2; shift 2
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
for r in $(seq 1 $R); do
  for lib in $LIBS; do
    BSG_LIBRARY=$PWD/$L/$lib AB_TAG=${lib%.so} timeout -k 10 120 python tools/ab_tree.py "$@" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
