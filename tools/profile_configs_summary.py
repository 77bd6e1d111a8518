"""Summarise tools/profile_configs.sh: per configuration the step kernel's rocprofv3
average duration, HBM bytes per launch (FETCH_SIZE doubled for gfx950, + WRITE_SIZE;
MI355X_MICROARCH.md HBM section), algorithmic bytes and the VALU counts.
    python3 tools/profile_configs_summary.py gpurun_out/profcfg_r03 r03
-> profiles/<tag>/configs_pmc.json and profiles/<tag>/configs_kernel_stats/*.csv"""
import csv
import glob
import json
import os
import shutil
import sys

# SURVEY.md §8(d) bytes per env-step: 2*N*10*8 + 4A + 4O + 6 + ceil(N^2/8) + ceil(N/8) + 4K
ALGO = {"vertical": lambda N: 2 * N * 80 + 4 * 1 + 4 * (4 + 7 * (N - 1)) + 6 + -(-N * N // 8) + -(-N // 8),
        "descent": lambda N: 160 + 4 + 16 + 6 + 1 + 1,
        "merge": lambda N: 2 * N * 80 + 8 + 160 + 6 + -(-N * N // 8) + -(-N // 8) + 20}

out, tag = sys.argv[1], sys.argv[2]
os.makedirs(f"profiles/{tag}/configs_kernel_stats", exist_ok=True)
res = {}
for d in sorted(glob.glob(out + "/*_*")):
    name = os.path.basename(d)
    kind, N, E = name.split("_")[0], int(name.split("_")[1]), int(name.split("_")[2])
    stats = list(csv.DictReader(open(glob.glob(d + "/trace/run_kernel_stats.csv")[0])))
    st = [r for r in stats if "step_kernel" in r["Name"]]
    top = max(st, key=lambda r: int(r["Calls"]))
    agg = {}
    for f in glob.glob(d + "/pmc_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    m = {k: sum(v[2:]) / max(len(v) - 2, 1) for k, v in agg.items()}     # skip reset + 1st step
    hbm = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
    avg = float(top["AverageNs"]) * 1e-9
    algo = ALGO[kind](N) * E
    f64 = sum(m[k] for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                             "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64"))
    res[name] = {"kernel": top["Name"], "envs": E, "num_ac": N, "calls": int(top["Calls"]),
                 "kernel_avg_us": avg * 1e6, "algorithmic_bytes_per_launch": algo,
                 "achieved_GBs": algo / avg / 1e9, "hbm_frac_of_8TBs": algo / avg / 8e12,
                 "hbm_bytes_per_launch_pmc": hbm, "traffic_over_algorithmic": hbm / algo,
                 "waves_per_launch": m.get("SQ_WAVES"), "valu_insts_per_launch": m["SQ_INSTS_VALU"],
                 "valu_f64_insts_per_launch": f64,
                 "valu_issue_frac_at_2p4ghz": (4 * f64 + 2 * (m["SQ_INSTS_VALU"] - f64)) / 1024
                                              / (avg * 2.4e9)}
    shutil.copy(glob.glob(d + "/trace/run_kernel_stats.csv")[0],
                f"profiles/{tag}/configs_kernel_stats/{name}.csv")
json.dump(res, open(f"profiles/{tag}/configs_pmc.json", "w"), indent=1)
print(json.dumps(res, indent=1))
