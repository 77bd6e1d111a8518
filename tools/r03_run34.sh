set -o pipefail
bash tools/gpu_round.sh r03g || { echo ROUND_FAILED; exit 1; }
timeout -k 10 900 bash tools/profile_configs.sh r03g > gpurun_out/profcfg_r03g.log 2>&1 || { echo PROFCFG_FAILED; tail -5 gpurun_out/profcfg_r03g.log; exit 1; }
tail -3 gpurun_out/profcfg_r03g.log
