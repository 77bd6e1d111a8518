set -o pipefail
bash tools/gpu_round.sh r03h || { echo ROUND_FAILED; exit 1; }
timeout -k 10 900 bash tools/profile_configs.sh r03h > gpurun_out/profcfg_r03h.log 2>&1 || { echo PROFCFG_FAILED; tail -5 gpurun_out/profcfg_r03h.log; exit 1; }
tail -3 gpurun_out/profcfg_r03h.log
