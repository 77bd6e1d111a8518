set -o pipefail
SKIP_PROF=1 bash tools/gpu_round.sh r03c || { echo ROUND_FAILED; exit 1; }
