set -o pipefail
mkdir -p gpurun_out/r03
export BSG_LIBRARY=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib/libbsg_stamps.so
for E in 512 2048; do
for v in "def:" "nolacd:BSG_LA_CD=0" "old:BSG_LA_CD=0 BSG_NO_FASTPATH=1"; do
  n=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 240 python -u tools/stamps.py $E 32 > gpurun_out/r03/st26_${n}_$E.txt 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/r03/st26_${n}_$E.txt; exit 1; }
done
done
for f in gpurun_out/r03/st26_*.txt; do echo "== $f"; sed -n 2,13p $f; grep -A7 "lookahead waves" $f; done
