"""Replay helpers: drive the batched CPU oracle over the golden episodes (all episodes of
a fixture as parallel envs) and collect per-step outputs aligned with the fixture."""
from __future__ import annotations

import numpy as np

from oracle import batched as ob
from oracle import bluesky_subset as bsx


def wind_from_golden(g):
    """The WindField a wind_* fixture was recorded with (None for the others)."""
    if "wind_lat" not in g:
        return None
    f = bsx.WindField()
    f.addpointvne(g["wind_lat"], g["wind_lon"], g["wind_vnorth"], g["wind_veast"],
                  g["wind_alt"] if "wind_alt" in g else None)
    return f


def _apply_wind(o, g):
    f = wind_from_golden(g)
    if f is not None:
        o.set_wind(f, augment_obs=True)


def replay_merge(g, autoreset=ob.AUTORESET_NONE):
    n_ep = len(g["length"])
    N = int(g["num_ac"])
    T = g["actions"].shape[1]
    o = ob.MergeOracle(n_ep, num_ac=N, autoreset=autoreset, compute_cd=False)
    _apply_wind(o, g)
    r0 = o.reset(spawn=g["spawn"])
    out = {"obs0": r0["obs"], "obs": [], "reward": [], "terminated": [], "truncated": [],
           "topk": [], "intr": [], "state": [], "info": []}
    for t in range(T):
        r = o.step(g["actions"][:, t])
        out["obs"].append(r["obs"]); out["reward"].append(r["reward"])
        out["terminated"].append(r["terminated"]); out["truncated"].append(r["truncated"])
        out["topk"].append(r["topk"])
        out["intr"].append(np.stack([(r["intr_mask"] >> np.uint64(i + 1)) & np.uint64(1)
                                     for i in range(N - 1)], 1).astype(np.int8))
        out["state"].append(np.stack([o.st.lat, o.st.lon, o.st.alt, o.st.hdg, o.st.tas,
                                      o.st.cas, o.st.vs], 1))
        inf = o.info()
        out["info"].append(np.stack([inf["total_reward"], inf["faf_reach"],
                                     inf["average_drift"], inf["total_intrusions"]], 1))
    return {k: (np.stack(v, 1) if k != "obs0" else v) for k, v in out.items()}


def replay_vertical(g, autoreset=ob.AUTORESET_NONE):
    n_ep = len(g["length"])
    N = int(g["num_ac"])
    T = g["actions"].shape[1]
    o = ob.VerticalOracle(n_ep, num_ac=N, autoreset=autoreset, compute_cd=False)
    _apply_wind(o, g)
    r0 = o.reset(spawn=g["spawn"])
    out = {"obs0": r0["obs"], "obs": [], "reward": [], "terminated": [], "truncated": [],
           "intr": [], "state": [], "info": []}
    for t in range(T):
        r = o.step(g["actions"][:, t])
        out["obs"].append(r["obs"]); out["reward"].append(r["reward"])
        out["terminated"].append(r["terminated"]); out["truncated"].append(r["truncated"])
        out["intr"].append(np.stack([(r["intr_mask"] >> np.uint64(i + 1)) & np.uint64(1)
                                     for i in range(N - 1)], 1).astype(np.int8))
        out["state"].append(np.stack([o.st.lat, o.st.lon, o.st.alt, o.st.hdg, o.st.tas,
                                      o.st.cas, o.st.vs], 1))
        inf = o.info()
        out["info"].append(np.stack([inf["total_reward"], inf["total_intrusions"],
                                     inf["final_altitude"]], 1))
    return {k: (np.stack(v, 1) if k != "obs0" else v) for k, v in out.items()}


def replay_descent(g, autoreset=ob.AUTORESET_NONE):
    n_ep = len(g["length"])
    T = g["actions"].shape[1]
    o = ob.DescentOracle(n_ep, autoreset=autoreset)
    _apply_wind(o, g)
    r0 = o.reset(spawn=g["spawn"])
    out = {"obs0": r0["obs"], "obs": [], "reward": [], "terminated": [], "truncated": [],
           "state": [], "info": []}
    for t in range(T):
        r = o.step(g["actions"][:, t])
        out["obs"].append(r["obs"]); out["reward"].append(r["reward"])
        out["terminated"].append(r["terminated"]); out["truncated"].append(r["truncated"])
        out["state"].append(np.stack([o.st.lat, o.st.lon, o.st.alt, o.st.hdg, o.st.tas,
                                      o.st.cas, o.st.vs], 1))
        inf = o.info()
        out["info"].append(np.stack([inf["total_reward"], inf["final_altitude"]], 1))
    return {k: (np.stack(v, 1) if k != "obs0" else v) for k, v in out.items()}


def replay_horizontal(g, autoreset=ob.AUTORESET_NONE):
    n_ep = len(g["length"])
    N = int(g["num_ac"])
    T = g["actions"].shape[1]
    o = ob.HorizontalOracle(n_ep, num_ac=N, autoreset=autoreset, compute_cd=False)
    _apply_wind(o, g)
    r0 = o.reset(spawn=g["spawn"])
    out = {"obs0": r0["obs"], "obs": [], "reward": [], "terminated": [], "truncated": [],
           "intr": [], "state": [], "info": []}
    for t in range(T):
        r = o.step(g["actions"][:, t])
        out["obs"].append(r["obs"]); out["reward"].append(r["reward"])
        out["terminated"].append(r["terminated"]); out["truncated"].append(r["truncated"])
        out["intr"].append(np.stack([(r["intr_mask"] >> np.uint64(i + 1)) & np.uint64(1)
                                     for i in range(N - 1)], 1).astype(np.int8))
        out["state"].append(np.stack([o.st.lat, o.st.lon, o.st.alt, o.st.hdg, o.st.tas,
                                      o.st.cas, o.st.vs], 1))
        inf = o.info()
        out["info"].append(np.stack([inf["total_reward"], inf["total_intrusions"],
                                     inf["average_drift"]], 1))
    out["wpt"] = np.stack([o.wpt_lat, o.wpt_lon], 1)
    return {k: (np.stack(v, 1) if k not in ("obs0", "wpt") else v) for k, v in out.items()}


def replay_static(g, autoreset=ob.AUTORESET_NONE):
    from oracle import batched_areas as oba
    n_ep = len(g["length"])
    T = g["actions"].shape[1]
    o = oba.StaticOracle(n_ep, autoreset=autoreset)
    _apply_wind(o, g)
    r0 = o.reset(spawn=g["spawn"])
    out = {"obs0": r0["obs"], "obs": [], "reward": [], "terminated": [], "truncated": [],
           "state": [], "info": []}
    geo = {"clat": o.clat.copy(), "clon": o.clon.copy(), "R": o.R.copy(),
           "wpt": np.stack([o.wlat, o.wlon], 1), "polys": [list(p) for p in o.polys]}
    for t in range(T):
        r = o.step(g["actions"][:, t])
        out["obs"].append(r["obs"]); out["reward"].append(r["reward"])
        out["terminated"].append(r["terminated"]); out["truncated"].append(r["truncated"])
        out["state"].append(np.stack([o.st.lat, o.st.lon, o.st.alt, o.st.hdg, o.st.tas,
                                      o.st.cas, o.st.vs], 1))
        inf = o.info()
        out["info"].append(np.stack([inf["total_reward"], inf["waypoint_reached"],
                                     inf["crashed"], inf["average_drift"]], 1))
    res = {k: (np.stack(v, 1) if k != "obs0" else v) for k, v in out.items()}
    res["geo"] = geo
    return res


def replay_sector(g, autoreset=ob.AUTORESET_NONE):
    from oracle import batched_areas as oba
    n_ep = len(g["length"])
    N = int(g["num_ac"])
    T = g["actions"].shape[1]
    o = oba.SectorOracle(n_ep, num_ac=N, autoreset=autoreset, compute_cd=False)
    _apply_wind(o, g)
    r0 = o.reset(spawn=g["spawn"])
    out = {"obs0": r0["obs"], "obs": [], "reward": [], "terminated": [], "truncated": [],
           "intr": [], "state": [], "info": []}
    for t in range(T):
        r = o.step(g["actions"][:, t])
        out["obs"].append(r["obs"]); out["reward"].append(r["reward"])
        out["terminated"].append(r["terminated"]); out["truncated"].append(r["truncated"])
        out["intr"].append(np.stack([(r["intr_mask"] >> np.uint64(i + 1)) & np.uint64(1)
                                     for i in range(N - 1)], 1).astype(np.int8))
        st = np.stack([o.st.lat, o.st.lon, o.st.alt, o.st.hdg, o.st.tas, o.st.cas, o.st.vs], 1)
        st = np.where(o.active()[:, None, :], st, 0.0)
        out["state"].append(st)
        inf = o.info()
        out["info"].append(np.stack([inf["total_reward"], inf["total_intrusions"],
                                     inf["average_drift"]], 1))
    return {k: (np.stack(v, 1) if k != "obs0" else v) for k, v in out.items()}


def replay_sequential(o, g, info_keys):
    """One env driven over the golden's consecutive episodes (reset from each spawn row,
    then the recorded steps) -- the goldens of the envs whose reset keeps a truncated
    episode's aircraft (descent_keep, plan*: make_golden.py gen_plan / keep_traffic)."""
    _apply_wind(o, g)
    n_ep, T = g["actions"].shape[:2]
    out = {k: np.zeros_like(g[k]) for k in ("obs0", "obs", "reward", "state", "info")}
    out["terminated"] = np.zeros_like(g["terminated"])
    out["truncated"] = np.zeros_like(g["truncated"])
    wpt = []
    for ep in range(n_ep):
        out["obs0"][ep] = o.reset(spawn=g["spawn"][ep:ep + 1])["obs"][0]
        if hasattr(o, "wpt_lat"):
            wpt.append(np.concatenate([np.ravel(o.wpt_lat[0]), np.ravel(o.wpt_lon[0])]))
        for t in range(int(g["length"][ep])):
            r = o.step(g["actions"][ep, t][None])
            out["obs"][ep, t] = r["obs"][0]
            out["reward"][ep, t] = r["reward"][0]
            out["terminated"][ep, t] = r["terminated"][0]
            out["truncated"][ep, t] = r["truncated"][0]
            out["state"][ep, t] = np.stack([o.st.lat, o.st.lon, o.st.alt, o.st.hdg, o.st.tas,
                                            o.st.cas, o.st.vs], 1)[0]
            inf = o.info()
            out["info"][ep, t] = [inf[k][0] for k in info_keys]
    if wpt:
        out["wpt"] = np.stack(wpt)
    return out


def replay_plan(g):
    o = ob.PlanWaypointOracle(1, autoreset=ob.AUTORESET_NONE, max_episode_steps=g["actions"].shape[1])
    return replay_sequential(o, g, ("total_reward", "waypoints_completed"))


def replay_descent_keep(g):
    o = ob.DescentOracle(1, autoreset=ob.AUTORESET_NONE, max_episode_steps=g["actions"].shape[1])
    return replay_sequential(o, g, ("total_reward", "final_altitude"))


def step_mask(g):
    """[n_ep, T] bool: steps inside each recorded episode."""
    T = g["actions"].shape[1]
    return np.arange(T)[None, :] < g["length"][:, None]
