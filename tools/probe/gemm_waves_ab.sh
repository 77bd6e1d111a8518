#!/bin/bash
# FusedSAC update time (tools/probe/sac_update_probe.py) with gemm256_kernel's K split over
# 4 / 8 / 16 waves (tools/_lib/libsacfused_w<N>.so), alternating.
set -euo pipefail
for r in 1 2; do
  for w in 4 8 16; do
    echo "w=$w run $r: $(SAC_FUSED_LIB=$PWD/tools/_lib/libsacfused_w$w.so timeout -k 10 120 python tools/probe/sac_update_probe.py 4 1 2>/dev/null | head -1)"
  done
done
