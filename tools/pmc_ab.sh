#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ab; mkdir -p $OUT
for v in cur skipown; do
 for c in "merge 32 4096 0 0" "merge 32 4096 1 0" "merge 32 4096 2 0"; do
  tag=${v}_$(echo $c | tr ' ' '_')
  BSG_LIBRARY=$PWD/build/variants/libbsg_$v.so timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $OUT/$tag -o run -- python3 tools/one_config.py $c 12 > /dev/null 2>&1 || echo "fail $tag"
 done
done
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/pmc_ab/*")):
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not agg: print(d, "none"); continue
    w = sum(agg["SQ_WAVES"]) / len(agg["SQ_WAVES"])
    m = {k: sum(v[2:]) / max(len(v) - 2, 1) for k, v in agg.items()}
    print(d.split("/")[-1], "per-wave: " + "  ".join(f"{k[8:]}={m[k]/w:.0f}" for k in sorted(m) if k != "SQ_WAVES"))
PY
