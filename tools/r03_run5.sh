set -o pipefail
mkdir -p gpurun_out/r03
echo "== default"; timeout -k 10 100 python tools/ablate.py descent_4096 descent_512 vert32_full_2048 2>&1 | grep -v amdgpu.ids
echo "== BSG_NO_FASTPATH=1"; BSG_NO_FASTPATH=1 timeout -k 10 100 python tools/ablate.py descent_4096 descent_512 vert32_full_2048 2>&1 | grep -v amdgpu.ids
