#!/bin/bash
# Compiler-flag sweep for the Merge step kernel (experiment builds, Merge only).
#   build (CPU container):  bash tools/flag_sweep.sh build
#   time  (GPU box):        bash tools/flag_sweep.sh run
set -euo pipefail
CS=bluesky-gym-hallucination_amd/csrc
OUT=build/variants
BASE="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -DBSG_ONLY_MERGE=1"
declare -A V
V[base]="-mllvm -disable-machine-licm"
V[maxilp]="-mllvm -disable-machine-licm -mllvm -amdgpu-sched-strategy=max-ilp"
V[bias0]="-mllvm -disable-machine-licm -mllvm -amdgpu-schedule-metric-bias=0"
V[nopostlicm]="-mllvm -disable-machine-licm -mllvm -disable-postra-machine-licm"
V[licm]=""
if [ "${1:-}" = build ]; then
  mkdir -p $OUT
  for k in "${!V[@]}"; do
    ( o=$OUT/obj_$k && mkdir -p $o && /opt/rocm/bin/hipcc $BASE ${V[$k]} -DBSG_KIND_TU=0 -c -o $o/k.o $CS/bsg_kernels.hip && /opt/rocm/bin/hipcc $BASE ${V[$k]} -x hip -c -o $o/d.o $CS/bsg_dispatch.cpp && /opt/rocm/bin/hipcc $BASE ${V[$k]} -x hip -c -o $o/a.o $CS/bsg_abi.cpp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libbsg_$k.so $o/k.o $o/d.o $o/a.o ) &
  done
  wait
  ls -la $OUT
else
  for k in "${!V[@]}"; do
    echo "== $k"
    BSG_LIBRARY=$PWD/$OUT/libbsg_$k.so ABLATE_OUT=gpurun_out/sweep_$k.json timeout -k 10 200 python tools/ablate.py merge32_full merge32_nocd
  done
fi
