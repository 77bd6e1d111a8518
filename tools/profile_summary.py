"""Summarise a tools/profile.sh run (rocprofv3 kernel-trace stats + separate PMC passes)
into profiles/<tag>/{kernel_stats.csv,pmc.json} and profiles/traffic.json.

Runs on the GPU box at the end of profile.sh and again in the build container on the
merged gpurun_out/prof_<tag>/ (only gpurun_out/ travels back):
    python3 tools/profile_summary.py gpurun_out/prof_r01 r01
"""
import csv
import glob
import json
import os
import shutil
import sys

out, tag = sys.argv[1], sys.argv[2]


def _compiler_vgprs(kernel):
    """VGPRs of `kernel` from the committed resource-usage remarks, or None."""
    try:
        lines = open(f"profiles/{tag}/resource_usage.txt").read().splitlines()
    except OSError:
        return None
    # "void bsg::step_kernel<0, 32, false, 1>(bsg::KParams)" -> "step_kernelILi0ELi32ELb0ELi1E"
    args = [a.strip() for a in kernel.split("<", 1)[1].split(">", 1)[0].split(",")]
    mangled = "step_kernelI" + "".join(
        ("Lb1E" if a == "true" else "Lb0E") if a in ("true", "false") else f"Li{a}E" for a in args)
    for i, ln in enumerate(lines):
        if ln.startswith("Function Name:") and mangled in ln:
            return int(lines[i + 1].split(":")[1])
    return None


os.makedirs(f"profiles/{tag}", exist_ok=True)
agg = {}
meta = None
for f in glob.glob(out + "/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            meta = (r["Grid_Size"], r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
m = {k: sum(v) / len(v) for k, v in agg.items()}
stats = {r["Name"]: r for r in csv.DictReader(open(out + "/trace/run_kernel_stats.csv"))}
k = [n for n in stats if "step_kernel" in n][0]
avg_ns = float(stats[k]["AverageNs"])
f64 = (m["SQ_INSTS_VALU_FMA_F64"] + m["SQ_INSTS_VALU_MUL_F64"] + m["SQ_INSTS_VALU_ADD_F64"]
       + m["SQ_INSTS_VALU_TRANS_F64"])
res = {
    "tag": tag, "kernel": k, "envs": 4096, "num_ac": 32, "grid": meta[0],
    # rocprofv3's VGPR_Count reads half the granulated allocation (208 -> 104); the compiler's
    # own count comes from -Rpass-analysis=kernel-resource-usage (profiles/<tag>/resource_usage.txt)
    "vgpr": _compiler_vgprs(k), "vgpr_rocprof_field": meta[1],
    "sgpr": meta[2], "lds_bytes": meta[3], "kernel_avg_ns_rocprof": avg_ns,
    "kernel_calls_rocprof": int(stats[k]["Calls"]),
    "fetch_size_kb": m["FETCH_SIZE"], "write_size_kb": m["WRITE_SIZE"],
    "hbm_bytes_per_launch": (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024,
    "hbm_correction": "gfx950 FETCH_SIZE counts half of coalesced read bytes (MI355X_MICROARCH.md "
                      "HBM): read side doubled; WRITE_SIZE as reported; KB = 1024 B",
    "valu_insts_per_launch": m["SQ_INSTS_VALU"], "valu_f64_insts_per_launch": f64,
    "waves_per_launch": m["SQ_WAVES"],
    # issue-cycle model: f64 VALU 4 cycles per wave64 instruction, other VALU 2 (SIMD-32)
    "valu_issue_cycles_per_simd": (4 * f64 + 2 * (m["SQ_INSTS_VALU"] - f64)) / 1024,
    "source": f"rocprofv3 --kernel-trace --stats and separate --pmc passes of "
              f"`bench.py --steps N --warmup 5` ({out})",
}
res["valu_issue_frac_at_2p4ghz"] = res["valu_issue_cycles_per_simd"] / (avg_ns * 1e-9 * 2.4e9)
shutil.copy(out + "/trace/run_kernel_stats.csv", f"profiles/{tag}/kernel_stats.csv")
json.dump(res, open(f"profiles/{tag}/pmc.json", "w"), indent=1)
json.dump({k2: res[k2] for k2 in ("envs", "num_ac", "kernel", "fetch_size_kb", "write_size_kb",
                                  "hbm_bytes_per_launch", "hbm_correction", "valu_insts_per_launch",
                                  "valu_f64_insts_per_launch", "valu_issue_cycles_per_simd",
                                  "kernel_avg_ns_rocprof", "source")},
          open("profiles/traffic.json", "w"), indent=1)
print(json.dumps(res, indent=1))
