"""Generate the golden vectors that pin the CPU oracle to the REFERENCE env code.

Run in the build container only (needs /root/reference):

    python tests/golden/make_golden.py

It imports the reference's own ``merge_env.py`` / ``vertical_cr_env.py`` /
``descent_env.py`` with stand-in modules for the absent packages (oracle/ref_harness.py)
and ``bluesky`` bound to the NumPy BlueSky-subset restatement, seeds Python ``random``
/ legacy ``np.random`` exactly as the reference envs consume them (merge_env.py:115-116,
150-151; vertical_cr_env.py:188-195,267-268; descent_env.py:170-171), drives seeded
action sequences and records, per step: observation (sorted-key flatten), reward,
terminated, TimeLimit truncation, info, top-K intruder indices (the env's argsort at
merge_env.py:196), the intrusion mask (merge_env.py:278-283 / vertical_cr_env.py:233-239)
and the post-step aircraft state.  Output: tests/golden/*.npz (data only).
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import batched as ob            # noqa: E402
from oracle import bluesky_subset as bsx    # noqa: E402
from oracle.ref_harness import load_reference_envs  # noqa: E402

STATE_FIELDS = ("lat", "lon", "alt", "hdg", "tas", "cas", "vs")


def flat(obs, keys):
    return np.concatenate([np.asarray(obs[k], np.float64).ravel() for k in keys])


def snap(bs):
    return np.stack([np.array(getattr(bs.traf, f), np.float64) for f in STATE_FIELDS], 0)


def gen_merge(bs, mods, num_ac, episodes, seed, max_steps=50):
    m = mods["merge"]
    m.NUM_AC = num_ac
    random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env = m.MergeEnv()
    K = m.NUM_AC_STATE
    rec = {k: [] for k in ("spawn", "obs0", "actions", "obs", "reward", "terminated",
                           "truncated", "topk", "intr", "state", "info", "length")}
    for ep in range(episodes):
        rng_copy = random.Random()
        rng_copy.setstate(random.getstate())
        spawn = ob.merge_spawn_from_python_random(rng_copy, num_ac)
        obs0, info0 = env.reset()
        acts = rng_act.uniform(-1, 1, (max_steps, 2))
        O, R, T, TR, TK, IN, ST, INF = [], [], [], [], [], [], [], []
        for t in range(max_steps):
            obs, rew, term, trunc, info = env.step(acts[t])
            trunc = (t + 1) >= max_steps            # gymnasium TimeLimit(50)
            lat, lon = bs.traf.lat, bs.traf.lon
            d = bs.tools.geo.kwikdist_matrix(lat[0], lon[0], lat[1:], lon[1:])
            topk = np.argsort(d)[:K] + 1
            _, di = bs.tools.geo.kwikqdrdist(lat[0], lon[0], lat[1:], lon[1:])
            O.append(flat(obs, ob.MERGE_OBS_KEYS)); R.append(rew); T.append(int(term))
            TR.append(trunc); TK.append(topk); IN.append(di < m.INTRUSION_DISTANCE)
            ST.append(snap(bs))
            INF.append([info["total_reward"], info["faf_reach"], info["average_drift"],
                        info["total_intrusions"]])
            if term or trunc:
                break
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, ob.MERGE_OBS_KEYS))
        rec["actions"].append(acts)
        rec["obs"].append(pad(O, (len(O[0]),), np.float64))
        rec["reward"].append(pad(R, (), np.float64))
        rec["terminated"].append(pad(T, (), np.int8))
        rec["truncated"].append(pad(TR, (), np.int8))
        rec["topk"].append(pad(TK, (K,), np.int32))
        rec["intr"].append(pad(IN, (num_ac - 1,), np.int8))
        rec["state"].append(pad(ST, ST[0].shape, np.float64))
        rec["info"].append(pad(INF, (4,), np.float64))
        rec["length"].append(L)
    out = {k: np.stack(v) if k != "length" else np.array(v) for k, v in rec.items()}
    out["num_ac"] = np.array(num_ac)
    out["seed"] = np.array(seed)
    out["fix"] = np.array([m.FIX_LAT, m.FIX_LON])
    return out


def gen_vertical(bs, mods, num_intruders, episodes, seed, max_steps=300):
    m = mods["vertical"]
    m.NUM_INTRUDERS = num_intruders
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env = m.VerticalCREnv()
    rec = {k: [] for k in ("spawn", "obs0", "actions", "obs", "reward", "terminated",
                           "truncated", "intr", "state", "info", "length")}
    for ep in range(episodes):
        rs = np.random.RandomState()
        rs.set_state(np.random.get_state())
        spawn = ob.vertical_spawn_from_np_random(
            rs, num_intruders, lambda a: float(bsx.vcas2tas(np.float64(m.AC_SPD), np.float64(a))))
        obs0, _ = env.reset()
        acts = rng_act.uniform(-1, 1, (max_steps, 1))
        O, R, T, TR, IN, ST, INF = [], [], [], [], [], [], []
        for t in range(max_steps):
            # snapshot state BEFORE a terminal step deletes the aircraft
            obs, rew, term, trunc, info = env.step(acts[t])
            trunc = (t + 1) >= max_steps
            O.append(flat(obs, ob.VERTICAL_OBS_KEYS)); R.append(rew); T.append(int(term))
            TR.append(trunc)
            INF.append([info["total_reward"], info["total_intrusions"], info["final_altitude"]])
            if term or trunc:
                ST.append(ST[-1] if ST else np.zeros((len(STATE_FIELDS), num_intruders + 1)))
                IN.append(np.zeros(num_intruders, bool))
                break
            ST.append(snap(bs))
            lat, lon, alt = bs.traf.lat, bs.traf.lon, bs.traf.alt
            _, di = bs.tools.geo.kwikqdrdist(lat[0], lon[0], lat[1:], lon[1:])
            IN.append((di < m.INTRUSION_DISTANCE) & (np.abs(alt[0] - alt[1:]) < m.VERTICAL_MARGIN))
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, ob.VERTICAL_OBS_KEYS))
        rec["actions"].append(acts)
        rec["obs"].append(pad(O, (len(O[0]),), np.float64))
        rec["reward"].append(pad(R, (), np.float64))
        rec["terminated"].append(pad(T, (), np.int8))
        rec["truncated"].append(pad(TR, (), np.int8))
        rec["intr"].append(pad(IN, (num_intruders,), np.int8))
        rec["state"].append(pad(ST, ST[0].shape, np.float64))
        rec["info"].append(pad(INF, (3,), np.float64))
        rec["length"].append(L)
    out = {k: np.stack(v) if k != "length" else np.array(v) for k, v in rec.items()}
    out["num_ac"] = np.array(num_intruders + 1)
    out["seed"] = np.array(seed)
    return out


def gen_horizontal(bs, mods, num_intruders, episodes, seed, max_steps=300):
    m = mods["horizontal"]
    m.NUM_INTRUDERS = num_intruders
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env = m.HorizontalCREnv()
    rec = {k: [] for k in ("spawn", "obs0", "actions", "obs", "reward", "terminated",
                           "truncated", "intr", "state", "info", "length", "wpt")}
    for ep in range(episodes):
        rs = np.random.RandomState()
        rs.set_state(np.random.get_state())
        spawn = ob.horizontal_spawn_from_np_random(rs, num_intruders)
        obs0, _ = env.reset()
        acts = rng_act.uniform(-1, 1, (max_steps, 1))
        O, R, T, TR, IN, ST, INF = [], [], [], [], [], [], []
        for t in range(max_steps):
            obs, rew, term, trunc, info = env.step(acts[t])
            trunc = (t + 1) >= max_steps
            O.append(flat(obs, ob.HORIZONTAL_OBS_KEYS)); R.append(rew); T.append(int(term))
            TR.append(trunc)
            INF.append([info["total_reward"], info["total_intrusions"], info["average_drift"]])
            if term:        # the env deleted every aircraft (horizontal_cr_env.py:119-122)
                ST.append(ST[-1] if ST else np.zeros((len(STATE_FIELDS), num_intruders + 1)))
                IN.append(np.zeros(num_intruders, bool))
                break
            ST.append(snap(bs))
            lat, lon = bs.traf.lat, bs.traf.lon
            _, di = bs.tools.geo.kwikqdrdist(lat[0], lon[0], lat[1:], lon[1:])
            IN.append(di < m.INTRUSION_DISTANCE)
            if trunc:
                break
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, ob.HORIZONTAL_OBS_KEYS))
        rec["actions"].append(acts)
        rec["obs"].append(pad(O, (len(O[0]),), np.float64))
        rec["reward"].append(pad(R, (), np.float64))
        rec["terminated"].append(pad(T, (), np.int8))
        rec["truncated"].append(pad(TR, (), np.int8))
        rec["intr"].append(pad(IN, (num_intruders,), np.int8))
        rec["state"].append(pad(ST, ST[0].shape, np.float64))
        rec["info"].append(pad(INF, (3,), np.float64))
        rec["length"].append(L)
        rec["wpt"].append([env.wpt_lat[0], env.wpt_lon[0]])
    out = {k: np.stack(v) if k != "length" else np.array(v) for k, v in rec.items()}
    out["num_ac"] = np.array(num_intruders + 1)
    out["seed"] = np.array(seed)
    return out


def gen_descent(bs, mods, episodes, seed, max_steps=300):
    m = mods["descent"]
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env = m.DescentEnv()
    rec = {k: [] for k in ("spawn", "obs0", "actions", "obs", "reward", "terminated",
                           "truncated", "state", "info", "length")}
    for ep in range(episodes):
        bs.traf.reset()   # reference reset() does not clear traffic (descent_env.py:162-182)
        rs = np.random.RandomState()
        rs.set_state(np.random.get_state())
        spawn = ob.descent_spawn_from_np_random(rs)
        obs0, _ = env.reset()
        acts = rng_act.uniform(-1, 1, (max_steps, 1))
        O, R, T, TR, ST, INF = [], [], [], [], [], []
        for t in range(max_steps):
            pre = snap(bs)
            obs, rew, term, trunc, info = env.step(acts[t])
            trunc = (t + 1) >= max_steps
            O.append(flat(obs, ob.DESCENT_OBS_KEYS)); R.append(rew); T.append(int(term))
            TR.append(trunc)
            INF.append([info["total_reward"], info["final_altitude"]])
            ST.append(snap(bs) if bs.traf.ntraf else pre)
            if term or trunc:
                break
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, ob.DESCENT_OBS_KEYS))
        rec["actions"].append(acts)
        rec["obs"].append(pad(O, (4,), np.float64))
        rec["reward"].append(pad(R, (), np.float64))
        rec["terminated"].append(pad(T, (), np.int8))
        rec["truncated"].append(pad(TR, (), np.int8))
        rec["state"].append(pad(ST, ST[0].shape, np.float64))
        rec["info"].append(pad(INF, (2,), np.float64))
        rec["length"].append(L)
    out = {k: np.stack(v) if k != "length" else np.array(v) for k, v in rec.items()}
    out["seed"] = np.array(seed)
    return out


def main():
    bs, mods = load_reference_envs()
    fn = mods["functions"]
    known = {
        "fix": np.array(fn.get_point_at_distance(52.36239301495972, 4.713195734579777, 200, 0)),
        "bound": np.array([fn.bound_angle_positive_negative_180(a)
                           for a in (190.0, -540.0, -190.0, 180.0, -180.0, 359.0, 0.0)]),
        "bound_in": np.array([190.0, -540.0, -190.0, 180.0, -180.0, 359.0, 0.0]),
    }
    np.savez_compressed(os.path.join(HERE, "functions_known.npz"), **known)
    jobs = [
        ("merge_N8", lambda: gen_merge(bs, mods, 8, 4, 0)),
        ("merge_N16", lambda: gen_merge(bs, mods, 16, 3, 1)),
        ("merge_N20", lambda: gen_merge(bs, mods, 20, 3, 2)),
        ("merge_N32", lambda: gen_merge(bs, mods, 32, 2, 3)),
        ("vertical_N6", lambda: gen_vertical(bs, mods, 5, 3, 4)),
        ("vertical_N32", lambda: gen_vertical(bs, mods, 31, 2, 5)),
        ("descent", lambda: gen_descent(bs, mods, 4, 6)),
        ("horizontal_N6", lambda: gen_horizontal(bs, mods, 5, 3, 7)),
        ("horizontal_N16", lambda: gen_horizontal(bs, mods, 15, 2, 8)),
    ]
    for name, job in jobs:
        out = job()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print(name, "episodes", len(out["length"]), "lengths", out["length"].tolist())


if __name__ == "__main__":
    main()
