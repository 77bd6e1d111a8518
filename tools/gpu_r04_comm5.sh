#!/bin/bash
# The per-step gather after the fence / priority change: sharded + lookahead GPU tests, the
# shard-size sweep, the host-API probe.
set -uo pipefail
OUT=gpurun_out/${1:-r04comm5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_lookahead.py -x -v --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_gather_sweep.py > "$OUT/gather_sweep.txt" 2>&1 || exit 1
timeout -k 10 200 tools/probe/hostapi_probe 28 > "$OUT/hostapi_probe.txt" 2>&1 || exit 1
