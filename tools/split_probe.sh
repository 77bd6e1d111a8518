#!/bin/bash
# VERDICT r04 item 3 (the headline split): compile-time register budgets of the roles a split
# of step_kernel<MERGE,32> would launch as separate kernels.  tools/probe/la_split_probe.hip
# instantiates the lookahead role (the intruders' substeps one step ahead) as a kernel of its
# own; the step kernel's instances come from bsg_kernels.hip itself.  Prints VGPRs / scratch /
# occupancy per kernel, and the lookahead kernel forced to 3 and 4 waves per SIMD.
# CPU only (hipcc cross-compiles gfx950).  Output: profiles/r05/split_resource_usage.txt
set -euo pipefail
cd "$(dirname "$0")/../bluesky-gym-hallucination_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -mllvm -disable-machine-licm -DBSG_KIND_TU=0"
show() { grep -E "Function Name|VGPRs:|Occupancy|ScratchSize|VGPRs Spill" | sed 's/.*remark: //;s/ \[-Rpass.*//'; }
tmp=$(mktemp -d)
for W in 0 3 4; do
  if [ "$W" = 0 ]; then cp ../../tools/probe/la_split_probe.hip la_split_probe_tmp.hip
  else sed "s/__launch_bounds__(64) void la_only_kernel/__launch_bounds__(64) __attribute__((amdgpu_waves_per_eu($W,$W))) void la_only_kernel/" \
         ../../tools/probe/la_split_probe.hip > la_split_probe_tmp.hip; fi
  echo "== lookahead role as its own kernel, waves_per_eu ${W/0/default}"
  /opt/rocm/bin/hipcc $F -c -o "$tmp/p.o" la_split_probe_tmp.hip -Rpass-analysis=kernel-resource-usage 2>&1 \
    | show | grep -A4 "la_only" || true
  if [ "$W" = 0 ]; then
    echo "== step_kernel<MERGE, 32> instances (LAK = false: the 4,096 headline; LAK = true: with the lookahead)"
    /opt/rocm/bin/hipcc $F -c -o "$tmp/p.o" la_split_probe_tmp.hip -Rpass-analysis=kernel-resource-usage 2>&1 \
      | show | grep -A4 "step_kernelILi0ELi32ELb0ELi1ELb" || true
  fi
done
rm -f la_split_probe_tmp.hip
rm -rf "$tmp"
