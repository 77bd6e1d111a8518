#!/bin/bash
# A/B of two builds of libbsg on one box, alternating (tools/ab_tree.py: Merge x 32 HIP-event
# time per step): bash tools/ab_lib.sh <lib A> <lib B> [rounds] [E ...]
set -uo pipefail
A=$1; B=$2; R=${3:-3}; shift 3 || shift $#
SIZES=${*:-512 1024 2048 4096}
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
for r in $(seq 1 $R); do
  for lib in $A $B; do
    BSG_LIBRARY=$PWD/$L/$lib AB_TAG=${lib%.so} timeout -k 10 120 python tools/ab_tree.py $SIZES 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
