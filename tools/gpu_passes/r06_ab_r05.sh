#!/bin/bash
# Round-5 library (ab_r05/: the aa6ab42 tree's package and libbsg.so, built in-tree, git-ignored)
# against this tree's, alternating on one box: did round 6 move the Merge shard / headline kernels?
# Make ab_r05/ first (CPU): git archive aa6ab42 | tar -x -C /tmp/r05 && make -j8 -C
# /tmp/r05/bluesky-gym-hallucination_amd/csrc && mkdir -p ab_r05/bluesky-gym-hallucination_amd &&
# cp -r /tmp/r05/bluesky-gym-hallucination_amd/bluesky_gym ab_r05/bluesky-gym-hallucination_amd/
set -uo pipefail
OUT=gpurun_out/r06ab; mkdir -p $OUT
for r in 1 2 3; do
  (cd ab_r05 && AB_TAG=r05 timeout -k 10 120 python ../tools/ab_tree.py 512 1024 2048 4096) >> $OUT/ab.log 2>&1 || exit 1
  AB_TAG=r06 timeout -k 10 120 python tools/ab_tree.py 512 1024 2048 4096 >> $OUT/ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/ab.log
