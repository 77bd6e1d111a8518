"""Extract the MergeEnv-v0 DDPG / TD3 training-log tails the saturated-policy pin uses
(tests/test_ref_logs.py::test_merge_saturated_policy, tests/test_gpu_ref_logs.py).

Run in the build container only (reads /root/reference):

    python tests/golden/extract_merge_logs.py

From episode 3 on both logs were flown by a saturated actor -- a constant (+-1, +1) action,
a circling ownship (average_drift 1.552 +- 0.011 over 40,000 episodes) -- and
every episode is truncated at 50 steps.  The fixture holds the last 1,000 episodes of each
log: average_drift, total_intrusions, total_reward (numbers only).  The actors themselves
are listed in the reference's .MISSING_LARGE_BLOBS.
Output: tests/golden/merge_logs.npz.
"""
from __future__ import annotations

import csv
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LOGS = "/root/reference/scripts/common/results/logs_backup/MergeEnv-v0"
KEYS = ("average_drift", "total_intrusions", "total_reward")


def main():
    out = {}
    for alg in ("DDPG", "TD3"):
        with open(os.path.join(LOGS, f"MergeEnv-v0_{alg}.csv")) as f:
            rows = list(csv.DictReader(f))
        ts = np.array([float(r["timesteps"]) for r in rows])
        length = np.diff(np.concatenate([[0.0], ts]))
        tail = rows[-1000:]
        assert (length[-1000:] == 50).all()            # every logged episode truncated at 50
        for k in KEYS:
            out[f"{alg.lower()}/{k}"] = np.array([float(r[k]) for r in tail])
        out[f"{alg.lower()}/episodes"] = np.array(len(rows))
    np.savez_compressed(os.path.join(HERE, "merge_logs.npz"), **out)
    for k, v in out.items():
        print(k, v.shape, float(np.mean(v)))


if __name__ == "__main__":
    main()
