set -o pipefail
mkdir -p gpurun_out/r03
export BSG_LIBRARY=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg_stamps.so
for E in 1024 2048; do
  STAMPS_KIND=vertical timeout -k 10 240 python -u tools/stamps.py $E 32 > gpurun_out/r03/st31_vert_$E.txt 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/r03/st31_vert_$E.txt; exit 1; }
  sed -n 2,13p gpurun_out/r03/st31_vert_$E.txt; grep -A6 "lookahead waves" gpurun_out/r03/st31_vert_$E.txt
done
