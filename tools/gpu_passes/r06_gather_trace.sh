#!/bin/bash
# Kernel traces of the 512-env shard with and without the fused per-step gather: the launch
# gaps and the RCCL kernel's own time (where the gather's ~5.7 us per step go)
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06gt; mkdir -p $OUT
for m in bare fused; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$m -o run -- python3 tools/gather_trace.py 512 300 $m > $OUT/$m.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for m in ("bare", "fused"):
    f = glob.glob(f"gpurun_out/r06gt/{m}/**/run_kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if "step_kernel" in r["Kernel_Name"]][-200:]
    t0 = int(ks[0]["Start_Timestamp"])
    others = [r for r in rows if "step_kernel" not in r["Kernel_Name"] and int(r["Start_Timestamp"]) >= t0]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(ks, ks[1:])]
    per = (int(ks[-1]["Start_Timestamp"]) - t0) / 1e3 / (len(ks) - 1)
    dur.sort(); gaps.sort()
    print(f"{m}: step period {per:.2f} us, kernel p50 {dur[len(dur)//2]:.2f} us, gap p50 {gaps[len(gaps)//2]:.2f} p90 {gaps[int(len(gaps)*.9)]:.2f} us")
    names = {}
    for r in others:
        n = r["Kernel_Name"][:70]
        names.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in names.items():
        v.sort()
        print(f"   other kernel {n}: n={len(v)} p50 {v[len(v)//2]:.2f} us")
PY
