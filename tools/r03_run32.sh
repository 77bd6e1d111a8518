set -o pipefail
SKIP_PROF=1 bash tools/gpu_round.sh r03f || { echo ROUND_FAILED; exit 1; }
bash tools/r03_run31.sh || exit 1
