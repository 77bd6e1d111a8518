set -o pipefail
bash tools/gpu_round.sh r03e || { echo ROUND_FAILED; exit 1; }
timeout -k 10 900 bash tools/profile_configs.sh r03e > gpurun_out/profcfg_r03e.log 2>&1 || { echo PROFCFG_FAILED; tail -5 gpurun_out/profcfg_r03e.log; exit 1; }
tail -3 gpurun_out/profcfg_r03e.log
