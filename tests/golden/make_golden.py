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

from oracle import areas as oa              # noqa: E402
from oracle import batched as ob            # noqa: E402
from oracle import batched_areas as oba     # noqa: E402
from oracle import bluesky_subset as bsx    # noqa: E402
from oracle.ref_harness import load_reference_envs  # noqa: E402

STATE_FIELDS = ("lat", "lon", "alt", "hdg", "tas", "cas", "vs")


def flat(obs, keys):
    return np.concatenate([np.asarray(obs[k], np.float64).ravel() for k in keys])


def snap(bs):
    return np.stack([np.array(getattr(bs.traf, f), np.float64) for f in STATE_FIELDS], 0)


def _wrap(mods, env, keys, wind):
    """Optionally wrap with the reference WindFieldWrapper (bluesky_gym/wrappers/wind.py)."""
    if wind is None:
        return env, tuple(keys)
    env = mods["wind"].WindFieldWrapper(env, augment_obs=True, **wind)
    return env, tuple(sorted(tuple(keys) + ("wind_u", "wind_v")))


def _step(env, a):
    """env.step; for a WindFieldWrapper, its step (wind.py:43-54) inlined so that the
    terminal step of the envs that delete their aircraft (vertical_cr_env.py:300-303,
    descent_env.py:201-204, horizontal_cr_env.py:119-122) -- where the reference wrapper
    raises IndexError in _get_wind_observation -- is recorded with NaN wind keys."""
    if not hasattr(env, "_get_wind_observation"):
        return env.step(a)
    out = env.env.step(a)
    try:
        wu, wv = env._get_wind_observation()
    except IndexError:
        wu = wv = np.nan
    obs = {**out[0], "wind_u": np.array([wu]), "wind_v": np.array([wv])}
    return (obs,) + tuple(out[1:])


def gen_merge(bs, mods, num_ac, episodes, seed, max_steps=50, wind=None):
    m = mods["merge"]
    m.NUM_AC = num_ac
    random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env, keys = _wrap(mods, m.MergeEnv(), ob.MERGE_OBS_KEYS, wind)
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
            obs, rew, term, trunc, info = _step(env, acts[t])
            trunc = (t + 1) >= max_steps            # gymnasium TimeLimit(50)
            lat, lon = bs.traf.lat, bs.traf.lon
            d = bs.tools.geo.kwikdist_matrix(lat[0], lon[0], lat[1:], lon[1:])
            topk = np.argsort(d)[:K] + 1
            _, di = bs.tools.geo.kwikqdrdist(lat[0], lon[0], lat[1:], lon[1:])
            O.append(flat(obs, keys)); R.append(rew); T.append(int(term))
            TR.append(trunc); TK.append(topk); IN.append(di < m.INTRUSION_DISTANCE)
            ST.append(snap(bs))
            INF.append([info["total_reward"], info["faf_reach"], info["average_drift"],
                        info["total_intrusions"]])
            if term or trunc:
                break
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, keys))
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


def gen_vertical(bs, mods, num_intruders, episodes, seed, max_steps=300, wind=None):
    m = mods["vertical"]
    m.NUM_INTRUDERS = num_intruders
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env, keys = _wrap(mods, m.VerticalCREnv(), ob.VERTICAL_OBS_KEYS, wind)
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
            obs, rew, term, trunc, info = _step(env, acts[t])
            trunc = (t + 1) >= max_steps
            O.append(flat(obs, keys)); R.append(rew); T.append(int(term))
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
        rec["obs0"].append(flat(obs0, keys))
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


def gen_horizontal(bs, mods, num_intruders, episodes, seed, max_steps=300, wind=None):
    m = mods["horizontal"]
    m.NUM_INTRUDERS = num_intruders
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env, keys = _wrap(mods, m.HorizontalCREnv(), ob.HORIZONTAL_OBS_KEYS, wind)
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
            obs, rew, term, trunc, info = _step(env, acts[t])
            trunc = (t + 1) >= max_steps
            O.append(flat(obs, keys)); R.append(rew); T.append(int(term))
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
        rec["obs0"].append(flat(obs0, keys))
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


def gen_descent(bs, mods, episodes, seed, max_steps=300, wind=None, keep_traffic=False):
    """keep_traffic: the traffic is cleared only before the first episode, as a driver of
    the reference env would see it -- after a truncation the next reset keeps KL001
    (descent_env.py:173 cre refused; the aircraft is only deleted on termination)."""
    m = mods["descent"]
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env, keys = _wrap(mods, m.DescentEnv(), ob.DESCENT_OBS_KEYS, wind)
    rec = {k: [] for k in ("spawn", "obs0", "actions", "obs", "reward", "terminated",
                           "truncated", "state", "info", "length")}
    for ep in range(episodes):
        if ep == 0 or not keep_traffic:
            bs.traf.reset()   # reference reset() does not clear traffic (descent_env.py:162-182)
        rs = np.random.RandomState()
        rs.set_state(np.random.get_state())
        spawn = ob.descent_spawn_from_np_random(rs)
        obs0, _ = env.reset()
        acts = rng_act.uniform(-1, 1, (max_steps, 1))
        O, R, T, TR, ST, INF = [], [], [], [], [], []
        for t in range(max_steps):
            pre = snap(bs)
            obs, rew, term, trunc, info = _step(env, acts[t])
            trunc = (t + 1) >= max_steps
            O.append(flat(obs, keys)); R.append(rew); T.append(int(term))
            TR.append(trunc)
            INF.append([info["total_reward"], info["final_altitude"]])
            ST.append(snap(bs) if bs.traf.ntraf else pre)
            if term or trunc:
                break
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, keys))
        rec["actions"].append(acts)
        rec["obs"].append(pad(O, (len(O[0]),), np.float64))
        rec["reward"].append(pad(R, (), np.float64))
        rec["terminated"].append(pad(T, (), np.int8))
        rec["truncated"].append(pad(TR, (), np.int8))
        rec["state"].append(pad(ST, ST[0].shape, np.float64))
        rec["info"].append(pad(INF, (2,), np.float64))
        rec["length"].append(L)
    out = {k: np.stack(v) if k != "length" else np.array(v) for k, v in rec.items()}
    out["seed"] = np.array(seed)
    return out


def _plan_greedy(obs):
    """Steer at the nearest unreached waypoint (drift from the obs' cos/sin terms)."""
    d = np.where(np.asarray(obs["waypoint_reached"]) == 0, np.asarray(obs["waypoint_distance"]), np.inf)
    k = int(np.argmin(d))
    drift = np.degrees(np.arctan2(obs["sin_difference"][k], obs["cos_difference"][k]))
    return np.array([np.clip(-drift / 45.0, -1.0, 1.0)])


def gen_plan(bs, mods, episodes, seed, max_steps=300, wind=None, greedy=False):
    """PlanWaypointEnv-v0 driven as one env instance over consecutive episodes (traffic
    cleared only before the first): truncated episodes hand their aircraft to the next
    (plan_waypoint_env.py:164 cre refused), terminated ones delete it (:189-193)."""
    m = mods["plan"]
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env, keys = _wrap(mods, m.PlanWaypointEnv(), ob.PLAN_OBS_KEYS, wind)
    rec = {k: [] for k in ("spawn", "obs0", "actions", "obs", "reward", "terminated",
                           "truncated", "state", "info", "length", "wpt", "state0")}
    bs.traf.reset()
    for ep in range(episodes):
        rs = np.random.RandomState()
        rs.set_state(np.random.get_state())
        spawn = ob.plan_spawn_from_np_random(rs)
        obs0, _ = env.reset()
        obs = obs0
        base = env.unwrapped if hasattr(env, "unwrapped") else env
        wpt = np.concatenate([np.asarray(base.wpt_lat, np.float64), np.asarray(base.wpt_lon, np.float64)])
        st0 = snap(bs)
        acts = rng_act.uniform(-1, 1, (max_steps, 1))
        O, R, T, TR, ST, INF = [], [], [], [], [], []
        for t in range(max_steps):
            pre = snap(bs)
            if greedy:
                acts[t] = _plan_greedy(obs)
            obs, rew, term, trunc, info = _step(env, acts[t])
            trunc = (t + 1) >= max_steps
            O.append(flat(obs, keys)); R.append(rew); T.append(int(term))
            TR.append(trunc)
            INF.append([info["total_reward"], info["waypoints_completed"]])
            ST.append(snap(bs) if bs.traf.ntraf else pre)
            if term or trunc:
                break
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, keys))
        rec["wpt"].append(wpt)
        rec["state0"].append(st0)
        rec["actions"].append(acts)
        rec["obs"].append(pad(O, (len(O[0]),), np.float64))
        rec["reward"].append(pad(R, (), np.float64))
        rec["terminated"].append(pad(T, (), np.int8))
        rec["truncated"].append(pad(TR, (), np.int8))
        rec["state"].append(pad(ST, ST[0].shape, np.float64))
        rec["info"].append(pad(INF, (2,), np.float64))
        rec["length"].append(L)
    out = {k: np.stack(v) if k != "length" else np.array(v) for k, v in rec.items()}
    out["seed"] = np.array(seed)
    return out


def gen_static(bs, mods, episodes, seed, max_steps=100):
    """StaticObstacleEnv (static_obstacle_env.py) with the legacy np.random seeded; records
    the obstacle geometry the reference built (pins the host spawn rows)."""
    m = mods["static"]
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env = m.StaticObstacleEnv()
    keys = oba.STATIC_OBS_KEYS
    rec = {k: [] for k in ("spawn", "obs0", "actions", "obs", "reward", "terminated",
                           "truncated", "state", "info", "length", "clat", "clon", "R",
                           "wpt", "poly_lat", "poly_lon", "nvert")}
    for ep in range(episodes):
        rs = np.random.RandomState()
        rs.set_state(np.random.get_state())
        spawn = oa.static_spawn_from_np_random(rs)
        obs0, _ = env.reset()
        acts = rng_act.uniform(-1, 1, (max_steps, 2))
        O, R, T, TR, ST, INF = [], [], [], [], [], []
        for t in range(max_steps):
            obs, rew, term, trunc, info = _step(env, acts[t])
            trunc = (t + 1) >= max_steps
            O.append(flat(obs, keys)); R.append(rew); T.append(int(term)); TR.append(trunc)
            ST.append(snap(bs))
            INF.append([info["total_reward"], info["waypoint_reached"], info["crashed"],
                        info["average_drift"]])
            if term or trunc:
                break
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, keys))
        rec["actions"].append(acts)
        rec["obs"].append(pad(O, (len(O[0]),), np.float64))
        rec["reward"].append(pad(R, (), np.float64))
        rec["terminated"].append(pad(T, (), np.int8))
        rec["truncated"].append(pad(TR, (), np.int8))
        rec["state"].append(pad(ST, ST[0].shape, np.float64))
        rec["info"].append(pad(INF, (4,), np.float64))
        rec["length"].append(L)
        rec["clat"].append(env.obstacle_centre_lat)
        rec["clon"].append(env.obstacle_centre_lon)
        rec["R"].append(env.obstacle_radius)
        rec["wpt"].append([env.wpt_lat[0], env.wpt_lon[0]])
        pl = np.zeros((oa.STATIC_NUM_OBSTACLES, oa.STATIC_VMAX))
        pn = np.zeros((oa.STATIC_NUM_OBSTACLES, oa.STATIC_VMAX))
        nv = []
        for o, verts in enumerate(env.obstacle_vertices):
            v = np.asarray(verts)
            pl[o, :len(v)], pn[o, :len(v)] = v[:, 0], v[:, 1]
            nv.append(len(v))
        rec["poly_lat"].append(pl); rec["poly_lon"].append(pn); rec["nvert"].append(nv)
    out = {k: np.stack(v) if k != "length" else np.array(v) for k, v in rec.items()}
    out["seed"] = np.array(seed)
    return out


def gen_sector(bs, mods, episodes, seed, N=32, max_steps=200):
    """SectorCREnv (sector_cr_env.py, density mode "normal") with np.random seeded."""
    m = mods["sector"]
    np.random.seed(seed)
    rng_act = np.random.default_rng(seed)
    env = m.SectorCREnv()
    keys = oba.SECTOR_OBS_KEYS
    rec = {k: [] for k in ("spawn", "obs0", "actions", "obs", "reward", "terminated",
                           "truncated", "state", "info", "length", "intr", "num_ac_ep")}
    for ep in range(episodes):
        rs = np.random.RandomState()
        rs.set_state(np.random.get_state())
        spawn = oa.sector_spawn_from_np_random(rs, N)
        obs0, _ = env.reset()
        assert env.num_ac == int(spawn[0])
        acts = rng_act.uniform(-1, 1, (max_steps, 2))
        O, R, T, TR, ST, INF, IN = [], [], [], [], [], [], []
        for t in range(max_steps):
            obs, rew, term, trunc, info = _step(env, acts[t])
            trunc = bool(trunc) or (t + 1) >= max_steps
            O.append(flat(obs, keys)); R.append(rew); T.append(int(term)); TR.append(trunc)
            st = np.zeros((len(STATE_FIELDS), N))
            st[:, :env.num_ac] = snap(bs)
            ST.append(st)
            lat, lon = bs.traf.lat, bs.traf.lon
            _, di = bs.tools.geo.kwikqdrdist(lat[0], lon[0], lat[1:], lon[1:])
            inn = np.zeros(N - 1, bool)
            inn[:env.num_ac - 1] = di < m.INTRUSION_DISTANCE
            IN.append(inn)
            INF.append([info["total_reward"], info["total_intrusions"], info["average_drift"]])
            if term or trunc:
                break
        L = len(O)
        pad = lambda a, shape, dt: np.concatenate([np.asarray(a, dt), np.zeros((max_steps - L,) + shape, dt)])
        rec["spawn"].append(spawn)
        rec["obs0"].append(flat(obs0, keys))
        rec["actions"].append(acts)
        rec["obs"].append(pad(O, (len(O[0]),), np.float64))
        rec["reward"].append(pad(R, (), np.float64))
        rec["terminated"].append(pad(T, (), np.int8))
        rec["truncated"].append(pad(TR, (), np.int8))
        rec["state"].append(pad(ST, ST[0].shape, np.float64))
        rec["info"].append(pad(INF, (3,), np.float64))
        rec["intr"].append(pad(IN, (N - 1,), np.int8))
        rec["length"].append(L)
        rec["num_ac_ep"].append(env.num_ac)
    out = {k: np.stack(v) if k != "length" else np.array(v) for k, v in rec.items()}
    out["num_ac"] = np.array(N)
    out["seed"] = np.array(seed)
    return out


# Wind fields for the WindFieldWrapper goldens (README of bluesky_gym/wrappers: a static
# field of 4 points; here also one placed on the Merge approach, a 3-D profile and a
# constant single point).
WIND_MERGE = dict(lat=np.array([52.5, 52.5, 54.2, 54.2]), lon=np.array([4.2, 5.3, 4.2, 5.3]),
                  vnorth=np.array([[16.0, 12.0, 14.0, 15.0]]), veast=np.array([[3.0, 7.0, 9.0, 4.0]]))
WIND_README = dict(lat=np.array([51.9, 51.9, 52.1, 52.1]), lon=np.array([3.9, 4.1, 3.9, 4.1]),
                   vnorth=np.array([[16.0, 12.0, 14.0, 15.0]]), veast=np.array([[3.0, 7.0, 9.0, 4.0]]))
WIND_3D = dict(lat=np.array([51.9, 51.9, 52.1, 52.1]), lon=np.array([3.9, 4.1, 3.9, 4.1]),
               vnorth=np.array([[2.0, -3.0, 4.0, 1.0], [16.0, 12.0, 14.0, 15.0], [30.0, 25.0, 28.0, 20.0]]),
               veast=np.array([[1.0, 2.0, -2.0, 0.5], [3.0, 7.0, 9.0, 4.0], [-10.0, -6.0, -8.0, -12.0]]),
               alt=np.array([0.0, 2000.0, 5000.0]))
WIND_ONE = dict(lat=52.0, lon=4.0, vnorth=np.array([[-12.0]]), veast=np.array([[8.0]]))
WINDS = {"merge": WIND_MERGE, "readme": WIND_README, "3d": WIND_3D, "one": WIND_ONE}


def wind_record(w):
    out = {"wind_lat": np.atleast_1d(np.asarray(w["lat"], np.float64)),
           "wind_lon": np.atleast_1d(np.asarray(w["lon"], np.float64)),
           "wind_vnorth": np.asarray(w["vnorth"], np.float64),
           "wind_veast": np.asarray(w["veast"], np.float64)}
    if w.get("alt") is not None:
        out["wind_alt"] = np.asarray(w["alt"], np.float64)
    return out


def gen_noisy_merge(bs, mods, num_ac, episodes, seed, noise, max_steps=50):
    """Reference NoisyObservationWrapper (wrappers/uncertainty.py) around MergeEnv: records
    the noisy observations (noise drawn from the global np.random in the env's dict order)."""
    m = mods["merge"]
    m.NUM_AC = num_ac
    random.seed(seed)
    np.random.seed(seed + 1000)
    rng_act = np.random.default_rng(seed)
    env = mods["uncertainty"].NoisyObservationWrapper(m.MergeEnv(), noise_level=noise)
    O0, O, L = [], [], []
    acts_all = []
    for ep in range(episodes):
        obs0, _ = env.reset()
        acts = rng_act.uniform(-1, 1, (max_steps, 2))
        acts_all.append(acts)
        OO = []
        for t in range(max_steps):
            obs, rew, term, trunc, info = env.step(acts[t])
            OO.append(flat(obs, ob.MERGE_OBS_KEYS))
            if term or (t + 1) >= max_steps:
                break
        O0.append(flat(obs0, ob.MERGE_OBS_KEYS))
        L.append(len(OO))
        O.append(np.concatenate([np.asarray(OO), np.zeros((max_steps - len(OO), len(OO[0])))]))
    return {"obs0": np.stack(O0), "obs": np.stack(O), "length": np.array(L),
            "actions": np.stack(acts_all), "num_ac": np.array(num_ac), "seed": np.array(seed),
            "noise": np.array(noise)}


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
        ("wind_merge_N16", lambda: {**gen_merge(bs, mods, 16, 3, 9, wind=WIND_MERGE),
                                    **wind_record(WIND_MERGE)}),
        ("wind_vertical_N6", lambda: {**gen_vertical(bs, mods, 5, 3, 10, wind=WIND_3D),
                                      **wind_record(WIND_3D)}),
        ("wind_descent", lambda: {**gen_descent(bs, mods, 3, 11, wind=WIND_ONE),
                                  **wind_record(WIND_ONE)}),
        ("static", lambda: gen_static(bs, mods, 3, 14)),
        ("descent_keep", lambda: gen_descent(bs, mods, 4, 16, max_steps=25, keep_traffic=True)),
        ("plan", lambda: gen_plan(bs, mods, 4, 17, max_steps=60)),
        ("plan_long", lambda: gen_plan(bs, mods, 2, 18)),
        ("plan_greedy", lambda: gen_plan(bs, mods, 4, 19, max_steps=200, greedy=True)),
        ("sector_N32", lambda: gen_sector(bs, mods, 3, 15)),
        ("noisy_merge_N8", lambda: gen_noisy_merge(bs, mods, 8, 2, 13, 0.2)),
        ("wind_horizontal_N6", lambda: {**gen_horizontal(bs, mods, 5, 2, 12, wind=WIND_README),
                                        **wind_record(WIND_README)}),
    ]
    only = set(sys.argv[1:])            # optional: regenerate just these names
    for name, job in jobs:
        if only and name not in only:
            continue
        out = job()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print(name, "episodes", len(out["length"]), "lengths", out["length"].tolist())


if __name__ == "__main__":
    main()
