#!/bin/bash
# Instruction-fetch / SQ stall counters of the bench kernel (one group per pass).
set -euo pipefail
OUT=gpurun_out/pmc_icache
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --skip-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d "$OUT/p1" -o run -- python3 bench.py $ARGS > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES --output-format csv -d "$OUT/p2" -o run -- python3 bench.py $ARGS > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_IFETCH_LEVEL SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_INSTS_VALU --output-format csv -d "$OUT/p3" -o run -- python3 bench.py $ARGS > /dev/null
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:30s} mean {sum(v)/len(v):.4g}  n={len(v)}")
PY
