set -o pipefail
mkdir -p gpurun_out/r03
L=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib
BSG_LIBRARY=$L/libbsg_stamps.so timeout -k 10 180 python tools/stamps.py 4096 32 > gpurun_out/r03/stamps_4096b.txt 2>&1 || { echo STAMPS_FAILED; tail gpurun_out/r03/stamps_4096b.txt; exit 1; }
grep -A40 "per-SIMD finish" gpurun_out/r03/stamps_4096b.txt
