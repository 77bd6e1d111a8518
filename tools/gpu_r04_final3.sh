#!/bin/bash
# Final round-4 pass after the spawn cache, the cruise re-check and the lookahead-free instance: the GPU suite,
# smoke, bench, rocprofv3 stats + PMC, per-config profiles and the per-step gather sweep.
set -uo pipefail
bash tools/gpu_round.sh r04h || exit 1
mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u tools/shard_gather_sweep.py > gpurun_out/r04h/gather_sweep.txt 2>&1 || exit 1
bash tools/profile_configs.sh r04h || exit 1
