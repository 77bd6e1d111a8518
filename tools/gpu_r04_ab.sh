#!/bin/bash
# A/B of experiment builds under tools/_var (timing only): bash tools/gpu_r04_ab.sh OUT cfg... -- lib...
set -uo pipefail
export TMPDIR=/tmp
bash tools/ab.sh "$@"
