"""MergeEnv-v0 under the saturated policy of the reference's DDPG / TD3 training logs.

From episode 3 on, ``logs_backup/MergeEnv-v0/MergeEnv-v0_{DDPG,TD3}.csv`` were flown by a
saturated actor: a constant (+-1, +1) action (HDG +-15 deg, SPD +20 m/s every RL step),
a circling ownship.  Every episode is truncated at 50 steps, so the per-episode
statistics (average_drift, total_intrusions, total_reward) are a distributional pin of
the sim layer: the intruders' LNAV stream, the ownship's speed envelope at 10,000 m.

    python tools/merge_saturated.py [--envs 2048] [--a0 1] [--a1 1] [--set NAME=VALUE ...]

``--set`` overrides a constant of oracle/bluesky_subset.py (sensitivity sweeps).
Test infrastructure: uses oracle/ only (tests/test_ref_logs.py holds the pinned case).
"""
from __future__ import annotations

import argparse
import csv
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import batched as ob            # noqa: E402
from oracle import bluesky_subset as bsx    # noqa: E402

LOGDIR = "/root/reference/scripts/common/results/logs_backup/MergeEnv-v0"


def log_tail(alg, first=2):
    rows = list(csv.DictReader(open(os.path.join(LOGDIR, f"MergeEnv-v0_{alg}.csv"))))[first:]
    return {k: np.array([float(r[k]) for r in rows]) for k in
            ("average_drift", "total_intrusions", "total_reward")}


def rollout(E, a0, a1, seed=11, steps=50, num_ac=20):
    o = ob.MergeOracle(E, num_ac=num_ac, seed=seed, compute_cd=False)
    o.reset()
    act = np.tile([a0, a1], (E, 1)).astype(np.float64)
    for _ in range(steps):
        r = o.step(act)
    assert r["truncated"].all()
    info = o.info()
    return {k: np.asarray(info[k], np.float64) for k in
            ("average_drift", "total_intrusions", "total_reward")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--a0", type=float, default=1.0)
    ap.add_argument("--a1", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--num-ac", type=int, default=20)
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    for s in a.set:
        k, v = s.split("=")
        setattr(ob if k.startswith("MERGE_") else bsx, k, float(v))
        print(f"set {k} = {v}")
    t = time.time()
    ours = rollout(a.envs, a.a0, a.a1, a.seed, num_ac=a.num_ac)
    print(f"rollout {a.envs} envs {time.time() - t:.1f} s")
    for alg in ("DDPG", "TD3"):
        lg = log_tail(alg)
        for k in ("average_drift", "total_intrusions", "total_reward"):
            x, y = ours[k], lg[k]
            se = np.hypot(x.std() / np.sqrt(len(x)), y.std() / np.sqrt(len(y)))
            print(f"{alg:4s} {k:17s} ours {x.mean():9.4f} sd {x.std():.4f}  log {y.mean():9.4f} "
                  f"sd {y.std():.4f} (n={len(y)})  z {(x.mean() - y.mean()) / se:+7.2f}")
        h0 = np.bincount(ours["total_intrusions"].astype(int), minlength=8)[:8] / len(x)
        h1 = np.bincount(lg["total_intrusions"].astype(int), minlength=8)[:8] / len(y)
        print("     P(intrusions=k) ours", np.round(h0, 3), "\n                      log ", np.round(h1, 3))


if __name__ == "__main__":
    main()
