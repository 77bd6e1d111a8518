#!/bin/bash
# Dynamic instruction counts per substep section: the substep probe built with PROBE_CUT=k
# (the substep returns at mark k), one rocprofv3 PMC pass per build (GPU box, repo root).
#   bash tools/probe/pmc_sections.sh [OUT]
set -uo pipefail
OUT=${1:-gpurun_out/pmc_sections}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/probe/substep_probe.py > "$OUT/state.log" 2>&1 || exit 1
for b in substep_probe_cut5 substep_probe_cut6 substep_probe_cut1 substep_probe_cut2 substep_probe_cut3 substep_probe_cut4 substep_probe; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES \
    --output-format csv -d "$OUT/$b" -o run -- tools/probe/$b gpurun_out/substep_state.bin > "$OUT/$b.log" 2>&1 || exit 1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
order = ["substep_probe_cut5", "substep_probe_cut6", "substep_probe_cut1", "substep_probe_cut2",
         "substep_probe_cut3", "substep_probe_cut4", "substep_probe"]
names = ["bearing (dl carry, qdr_x_t)", "far test + near block", "(LNAV end)", "speed / limits / airspeed",
         "turn", "heading sin/cos", "vertical + position + lat carry"]
keys = ["SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
        "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_SALU", "SQ_WAVES"]
tot = {}
for b in order:
    agg = collections.defaultdict(float)
    for f in glob.glob(f"{out}/{b}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "probe" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    tot[b] = agg
waves = tot["substep_probe"].get("SQ_WAVES", 1.0) or 1.0
print(f"per wave per substep (10 substeps, {waves:.0f} waves incl. reps); cumulative cuts, then differences")
prev = {k: 0.0 for k in keys}
for b, n in zip(order, names):
    cur = {k: tot[b].get(k, 0.0) / waves / 10 for k in keys}
    d = {k: cur[k] - prev[k] for k in keys}
    print(f"{n:34s} VALU {d['SQ_INSTS_VALU']:7.1f}  f64 fma {d['SQ_INSTS_VALU_FMA_F64']:6.1f} mul {d['SQ_INSTS_VALU_MUL_F64']:6.1f} "
          f"add {d['SQ_INSTS_VALU_ADD_F64']:6.1f} trans {d['SQ_INSTS_VALU_TRANS_F64']:5.1f}  SALU {d['SQ_INSTS_SALU']:6.1f}")
    prev = cur
print(f"{'total':34s} VALU {prev['SQ_INSTS_VALU']:7.1f}")
PY
