set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 500 bash tools/profile.sh r03 > gpurun_out/r03/profile.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r03/profile.log; exit 1; }
tail -3 gpurun_out/r03/profile.log
timeout -k 10 650 bash tools/profile_configs.sh r03 > gpurun_out/r03/profile_configs.log 2>&1 || { echo PROFCFG_FAILED; tail -20 gpurun_out/r03/profile_configs.log; exit 1; }
tail -6 gpurun_out/r03/profile_configs.log
