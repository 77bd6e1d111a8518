#!/bin/bash
# where Descent's extra reads come from.  The same Descent 4096 workload
# (tools/one_config.py) on the product library (seven-wave pipeline, step_kernel<DESCENT,1,
# false,7>) and on libbsg_dc1.so (make descent-nocoop: the one-wave instance), each counter
# group in its own rocprofv3 pass: HBM bytes (FETCH_SIZE / WRITE_SIZE), the vector-memory side
# of L2 (TCP_TCC_*), the instruction / scalar caches (SQC_*) and the instruction counts.
# Usage (GPU box, repo root): bash tools/pmc_descent_ab.sh [outdir]
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_descent_ab}
mkdir -p "$OUT"
L=bluesky-gym-hallucination_amd/bluesky_gym/_lib
rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
  "SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_DCACHE_REQ SQC_DCACHE_MISSES"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_IFETCH"
)
for lib in libbsg.so libbsg_dc1.so; do
  tag=${lib%.so}
  BSG_LIBRARY=$PWD/$L/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag/trace" -o run \
    -- python3 tools/one_config.py descent 1 4096 30 0 40 > /dev/null 2>"$OUT/$tag.trace.err"
  rc=$?; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
  k=0
  for c in "${PASSES[@]}"; do
    k=$((k + 1))
    BSG_LIBRARY=$PWD/$L/$lib timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv \
      -d "$OUT/$tag/p$k" -o run -- python3 tools/one_config.py descent 1 4096 30 0 24 > /dev/null 2>"$OUT/$tag.p$k.err"
    rc=$?
    echo "$tag pass $k ($c): rc=$rc"
    [ $rc -eq 137 ] && exit $rc
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
res = {}
for tag in ("libbsg", "libbsg_dc1"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{tag}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    # per launch, the first launches (reset, priming) left out
    res[tag] = {k: sum(v[4:]) / max(len(v) - 4, 1) for k, v in agg.items()}
    names = set()
    for f in glob.glob(f"{out}/{tag}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                names.add(r["Kernel_Name"][:60])
    res[tag]["kernels"] = sorted(names)
json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
