set -o pipefail
mkdir -p gpurun_out/r03
export BSG_LIBRARY=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg_stamps.so
for E in 512 2048; do
  timeout -k 10 240 python -u tools/stamps.py $E 32 > gpurun_out/r03/stamps_la_$E.txt 2>&1 || { echo STAMPS_FAILED $E; tail -20 gpurun_out/r03/stamps_la_$E.txt; exit 1; }
done
unset BSG_LIBRARY
bash tools/gpu_round.sh r03d || { echo ROUND_FAILED; exit 1; }
