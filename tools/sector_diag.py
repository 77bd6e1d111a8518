"""SectorCREnv-v0: where the oracle's rollouts of the reference's SAC / PPO actors leave
their training logs.  Prints the episode-length histogram, drift by
length bucket and intrusions of ours next to the log's last 1,000 episodes.

    python tools/sector_diag.py [--tag sector|sector_ppo] [--envs 200] [--no-intruders]
                                [--set NAME=VALUE ...]

``--no-intruders`` zeroes the intruders' speed and moves them far away, isolating the
ownship.  ``--set`` overrides an oracle/bluesky_subset.py constant.  Test infrastructure:
oracle/ and tests/ref_policy.py only.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import ref_policy as sp                      # noqa: E402
from oracle import batched_areas as oba      # noqa: E402
from oracle import bluesky_subset as bsx     # noqa: E402

BUCKETS = ((0, 10), (10, 20), (20, 30), (30, 60), (60, 1000))
HIST = [0, 5, 10, 15, 20, 25, 30, 40, 60, 100, 400]


def rollout(tag, E, seed=0, horizon=400, spd_scale=1.0, hdg_scale=1.0, flip=(), af=5, dt=1.0):
    W = sp.load()
    o = oba.SectorOracle(E, seed=5, compute_cd=False, action_frequency=af, simdt=dt)
    rng = None if sp.alg_of(W, tag) == "ddpg" else np.random.default_rng(seed)
    obs = o.reset()["obs"]
    ndone = np.zeros(E, np.int64)
    length = np.zeros(E)
    rec = {k: np.full(E, np.nan) for k in sp.LOG_KEYS["sector"]}
    tas, acts = [], []
    for _ in range(horizon):
        ob_in = obs.copy()
        for c in flip:
            ob_in[:, c] = -ob_in[:, c]
        act = sp.actor_np(W, tag, ob_in, rng)
        act = act * np.array([hdg_scale, spd_scale])
        tas.append(o.st.tas[:, 0][ndone == 0].copy())
        acts.append(act[ndone == 0].copy())
        r = o.step(act)
        obs = r["obs"]
        live = (ndone == 0) & ~r["was_reset"]
        length[live] += 1
        d = (r["terminated"] | r["truncated"]) & ~r["was_reset"]
        info = o.info()
        for k in rec:
            rec[k][d & live] = np.asarray(info[k], np.float64)[d & live]
        ndone += d
        if (ndone > 0).all():
            break
    rec["length"] = length
    tas, acts = np.concatenate(tas), np.concatenate(acts)
    print(f"ownship TAS pct {np.percentile(tas, [1, 10, 50, 90, 99])}")
    print(f"action mean {acts.mean(0)} |a|>0.95 frac {(np.abs(acts) > 0.95).mean(0)}")
    print(f"action[1] hist {np.histogram(acts[:, 1], bins=8, range=(-1, 1))[0] / len(acts)}")
    return W, rec


def report(name, L, d, I):
    print(f"{name:5s} len {L.mean():7.2f} pct {np.percentile(L, [5, 25, 50, 75, 95])} "
          f"drift {np.nanmean(d):.4f} intr {np.nanmean(I):.3f}")
    print(f"      len hist {np.histogram(L, bins=HIST)[0] / len(L)}")
    print("      drift by length: " + "  ".join(
        f"[{lo},{hi}) {np.nanmean(d[(L >= lo) & (L < hi)]):.3f}"
        for lo, hi in BUCKETS if ((L >= lo) & (L < hi)).any()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="sector")
    ap.add_argument("--envs", type=int, default=200)
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--spd-scale", type=float, default=1.0, help="scale the actor's speed action")
    ap.add_argument("--hdg-scale", type=float, default=1.0, help="scale the actor's heading action")
    ap.add_argument("--flip", default="", help="comma list of obs columns negated for the actor")
    ap.add_argument("--af", type=int, default=5, help="ACTION_FREQUENCY (sector_cr_env.py:31: 5)")
    ap.add_argument("--dt", type=float, default=1.0, help="DT (sector_cr_env.py:77: 'DT 1')")
    a = ap.parse_args()
    for s in a.set:
        k, v = s.split("=")
        setattr(oba if k.startswith(("C_", "S_")) else bsx, k, float(v))
        print(f"set {k} = {v}")
    t = time.time()
    flip = tuple(int(c) for c in a.flip.split(',') if c)
    W, rec = rollout(a.tag, a.envs, spd_scale=a.spd_scale, hdg_scale=a.hdg_scale, flip=flip,
                     af=a.af, dt=a.dt)
    print(f"rollout {a.envs} envs {time.time() - t:.1f} s")
    log = sp.log_stats(W, a.tag)
    report("ours", rec["length"], rec["average_drift"], rec["total_intrusions"])
    report("log", log["length"], log["average_drift"], log["total_intrusions"])


if __name__ == "__main__":
    main()
