#!/bin/bash
# Round-6 GPU pass 1: the new learner-reduce tests, stamps of the C4 shards, the device z of
# the Merge CAS-100 statistics over seeds, the Descent counter A/B, the C5 bench at one rank
# over RCCL.  Every step under its own time limit; stops at the first failure.
set -uo pipefail
OUT=gpurun_out/r06a
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 4 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
step tests 600 python -u -m pytest tests/test_gpu_sac_adam.py tests/test_gpu_bench_contract.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
L=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib
for e in 512 1024 2048; do
  BSG_LIBRARY=$L/libbsg_stamps.so step stamps_$e 120 python -u tools/stamps.py $e 32 || exit 1
done
step merge_sat_z 300 python -u tools/merge_sat_z.py device || exit 1
step c5_rccl 300 python -u bench.py --workload descent-sac --steps 200 --warmup 20 || exit 1
step c5_noreduce 300 python -u bench.py --workload descent-sac --steps 200 --warmup 20 --learner-reduce torch || exit 1
step pmc_descent 600 bash tools/pmc_descent_ab.sh $OUT/pmc_descent_ab || exit 1
