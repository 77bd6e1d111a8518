#!/bin/bash
# Merge-only experiment builds of several kernel source trees for A/B timing (for flag
# variants of this tree, make -C bluesky-gym-hallucination_amd/csrc OUT=... OBJ_TAG=...
# CXXFLAGS_EXTRA=... / ILP_FLAGS=... and tools/ab_libs.sh are simpler).
#   build (CPU container):  bash tools/variants.sh build NAME=SRC_CSRC_DIR ...
#   time  (GPU box):        bash tools/variants.sh run NAME ...
set -euo pipefail
OUT=build/variants
# (the Makefile's flags for MergeEnv's units, ILP_FLAGS, unless ILP is set)
ILP=${ILP--mllvm -amdgpu-sched-strategy=max-ilp -DBSG_WAVES_PER_EU=2}
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -mllvm -disable-machine-licm -DBSG_ONLY_MERGE=1 $ILP ${XFLAGS:-}"
mode=$1; shift
if [ "$mode" = build ]; then
  mkdir -p $OUT
  for kv in "$@"; do
    k=${kv%%=*}; d=${kv#*=}; x=""
    case "$d" in *:*) x=${d#*:}; d=${d%%:*};; esac
    ( o=$OUT/obj_$k && mkdir -p $o && /opt/rocm/bin/hipcc $FLAGS $x -DBSG_KIND_TU=0 -c -o $o/k.o $d/bsg_kernels.hip && /opt/rocm/bin/hipcc $FLAGS $x -DBSG_MERGE_NL_TU=1 -c -o $o/nl.o $d/bsg_kernels.hip && /opt/rocm/bin/hipcc $FLAGS $x -x hip -c -o $o/d.o $d/bsg_dispatch.cpp && /opt/rocm/bin/hipcc $FLAGS $x -x hip -c -o $o/a.o $d/bsg_abi.cpp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libbsg_$k.so $o/k.o $o/nl.o $o/d.o $o/a.o build/obj/bsg_comm.o build/obj/bsg_policy.o -ldl ) &
  done
  wait
  ls -la $OUT
else
  for k in "$@"; do
    echo "== $k"
    BSG_LIBRARY=$PWD/$OUT/libbsg_$k.so ABLATE_OUT=gpurun_out/var_$k.json timeout -k 10 200 python tools/ablate.py ${ABL:-merge32_full merge32_nocd}
  done
fi
