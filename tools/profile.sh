#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes for the bench workload.
# Run on the GPU box from the repo root:  bash tools/profile.sh r01
# Writes gpurun_out/prof_<tag>/ and the summaries profiles/<tag>/{kernel_stats.csv,pmc.json}.
set -euo pipefail
TAG=${1:-r01}
STEPS=${STEPS:-50}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT" "profiles/$TAG"
export TMPDIR=/tmp
B="python3 bench.py --steps $STEPS --warmup 5 --skip-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B > "$OUT/bench_trace.json"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $B > /dev/null
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- $B > /dev/null
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/pmc_valu" -o run -- $B > /dev/null
cp "$OUT/trace/run_kernel_stats.csv" "profiles/$TAG/kernel_stats.csv"
python3 - "$OUT" "$TAG" <<'PY'
import csv, glob, json, sys
out, tag = sys.argv[1], sys.argv[2]
agg = {}
for f in glob.glob(out + "/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            meta = (r["Grid_Size"], r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
m = {k: sum(v) / len(v) for k, v in agg.items()}
stats = {r["Name"]: r for r in csv.DictReader(open(out + "/trace/run_kernel_stats.csv"))}
k = [n for n in stats if "step_kernel" in n][0]
avg_ns = float(stats[k]["AverageNs"])
f64 = m["SQ_INSTS_VALU_FMA_F64"] + m["SQ_INSTS_VALU_MUL_F64"] + m["SQ_INSTS_VALU_ADD_F64"] + m["SQ_INSTS_VALU_TRANS_F64"]
res = {
    "tag": tag, "kernel": k, "envs": 4096, "num_ac": 32, "grid": meta[0], "vgpr": meta[1],
    "sgpr": meta[2], "lds_bytes": meta[3], "kernel_avg_ns_rocprof": avg_ns,
    "fetch_size_kb": m["FETCH_SIZE"], "write_size_kb": m["WRITE_SIZE"],
    "hbm_bytes_per_launch": (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024,
    "hbm_correction": "gfx950 FETCH_SIZE counts half of coalesced read bytes (MI355X_MICROARCH.md HBM): read side doubled; WRITE_SIZE as reported; KB = 1024 B",
    "valu_insts_per_launch": m["SQ_INSTS_VALU"], "valu_f64_insts_per_launch": f64,
    "waves_per_launch": m["SQ_WAVES"],
    # issue-cycle model: f64 VALU 4 cycles per wave64 instruction, other VALU 2 (SIMD-32)
    "valu_issue_cycles_per_simd": (4 * f64 + 2 * (m["SQ_INSTS_VALU"] - f64)) / 1024,
    "source": f"rocprofv3 --kernel-trace --stats and separate --pmc passes of `bench.py --steps N --warmup 5` ({out})",
}
res["valu_issue_frac_at_2p4ghz"] = res["valu_issue_cycles_per_simd"] / (avg_ns * 1e-9 * 2.4e9)
json.dump(res, open(f"profiles/{tag}/pmc.json", "w"), indent=1)
json.dump({k2: res[k2] for k2 in ("envs", "num_ac", "kernel", "fetch_size_kb", "write_size_kb",
                                  "hbm_bytes_per_launch", "hbm_correction", "valu_insts_per_launch",
                                  "valu_f64_insts_per_launch", "valu_issue_cycles_per_simd",
                                  "kernel_avg_ns_rocprof", "source")},
          open("profiles/traffic.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
