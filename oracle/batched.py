"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- batched NumPy restatement of the env layer.

Restates, for E independent envs at once ([E, N] structure-of-arrays), what the
reference env classes compute per env:

* ``MergeOracle``     -- bluesky_gym/envs/merge_env.py:103-293
* ``VerticalOracle``  -- bluesky_gym/envs/vertical_cr_env.py:113-305
* ``DescentOracle``   -- bluesky_gym/envs/descent_env.py:89-206
* ``HorizontalOracle`` -- bluesky_gym/envs/horizontal_cr_env.py:82-275
* ``PlanWaypointOracle`` -- bluesky_gym/envs/plan_waypoint_env.py:86-227

plus Gymnasium's ``TimeLimit`` (bluesky_gym/__init__.py:9,27,45) and the two vector
autoreset conventions (Gymnasium NEXT_STEP, SB3 SAME_STEP).  The simulator arithmetic
comes from ``oracle.bluesky_subset``.  Pinned against the reference's own env code by
``tests/golden/*.npz`` (see tests/golden/make_golden.py, tests/test_oracle_golden.py).

This module is the checker for ``libbsg.so``; the product never imports it.
"""
from __future__ import annotations

import math

import numpy as np

from . import bluesky_subset as bsx
from . import philox

NM2KM = 1.852
MPS2KT = 1.94384

AUTORESET_NONE = 0
AUTORESET_NEXT_STEP = 1
AUTORESET_SAME_STEP = 2

# ---- merge_env.py:13-46 ---------------------------------------------------------------
MERGE_DISTANCE_MARGIN = 10
MERGE_REACH_REWARD = 1
MERGE_DRIFT_PENALTY = -0.1
MERGE_INTRUSION_PENALTY = -1
MERGE_INTRUSION_DISTANCE = 4
MERGE_SPAWN_DISTANCE_MIN, MERGE_SPAWN_DISTANCE_MAX = 50, 200
MERGE_INTRUDER_DISTANCE_MIN, MERGE_INTRUDER_DISTANCE_MAX = 20, 500
MERGE_D_HEADING = 15
MERGE_D_SPEED = 20
MERGE_AC_SPD = 100
MERGE_ALT = 10000
RWY_LAT = 52.36239301495972
RWY_LON = 4.713195734579777
FIX_LAT, FIX_LON = (float(v) for v in bsx.get_point_at_distance(RWY_LAT, RWY_LON, 200, 0))

# ---- vertical_cr_env.py:12-45 / descent_env.py:10-30 -----------------------------------
V_INTRUSION_PENALTY = -50
V_ALT_DIF_REWARD_SCALE = -5 / 3000
V_CRASH_PENALTY = -100
V_RWY_ALT_DIF_REWARD_SCALE = -50 / 3000
V_INTRUSION_DISTANCE = 5
V_VERTICAL_MARGIN = 1000 * 0.3048
ALT_MEAN, ALT_STD = 1500, 3000
VZ_MEAN, VZ_STD = 0, 5
RWY_DIS_MEAN, RWY_DIS_STD = 100, 200
DEFAULT_RWY_DIS = 200
V_RWY_LAT, V_RWY_LON = 52, 4
ACTION_2_MS = 12.5
ALT_MIN, ALT_MAX = 2000, 4000
TARGET_ALT_DIF = 500
V_AC_SPD = 150
V_INTRUSION_DISTANCE_INT = 5   # randint upper bound for cpa (vertical_cr_env.py:189)

MERGE_OBS_KEYS = ("airspeed", "cos(drift)", "cos(track)", "distances", "faf_reached",
                  "sin(drift)", "sin(track)", "vx_r", "vy_r", "waypoint_dist", "x_r", "y_r")
VERTICAL_OBS_KEYS = ("altitude", "altitude_difference", "cos_difference_pos",
                     "intruder_distance", "runway_distance", "sin_difference_pos",
                     "target_altitude", "vz", "x_difference_speed", "y_difference_speed",
                     "z_difference_speed")
DESCENT_OBS_KEYS = ("altitude", "runway_distance", "target_altitude", "vz")
PLAN_OBS_KEYS = ("cos_difference", "sin_difference", "waypoint_distance", "waypoint_reached")
HORIZONTAL_OBS_KEYS = ("cos_difference_pos", "cos_drift", "intruder_distance",
                       "sin_difference_pos", "sin_drift", "waypoint_distance",
                       "x_difference_speed", "y_difference_speed")

# ---- horizontal_cr_env.py:11-30 ------------------------------------------------------------
H_DISTANCE_MARGIN = 5
H_REACH_REWARD = 1
H_DRIFT_PENALTY = -0.1
H_INTRUSION_PENALTY = -1
H_INTRUSION_DISTANCE = 5
H_WAYPOINT_DISTANCE_MIN, H_WAYPOINT_DISTANCE_MAX = 100, 150
H_D_HEADING = 45
H_AC_SPD = 150


def merge_obs_sizes(k):
    return {"airspeed": 1, "cos(drift)": 1, "cos(track)": k, "distances": k,
            "faf_reached": 1, "sin(drift)": 1, "sin(track)": k, "vx_r": k, "vy_r": k,
            "waypoint_dist": 1, "x_r": k, "y_r": k}


def vertical_obs_sizes(ni):
    return {"altitude": 1, "altitude_difference": ni, "cos_difference_pos": ni,
            "intruder_distance": ni, "runway_distance": 1, "sin_difference_pos": ni,
            "target_altitude": 1, "vz": 1, "x_difference_speed": ni,
            "y_difference_speed": ni, "z_difference_speed": ni}


def horizontal_obs_sizes(ni):
    return {"cos_difference_pos": ni, "cos_drift": 1, "intruder_distance": ni,
            "sin_difference_pos": ni, "sin_drift": 1, "waypoint_distance": 1,
            "x_difference_speed": ni, "y_difference_speed": ni}


def descent_obs_sizes():
    return {k: 1 for k in DESCENT_OBS_KEYS}


# ---- plan_waypoint_env.py:11-23 --------------------------------------------------------------
P_DISTANCE_MARGIN = 5
P_WAYPOINT_DISTANCE_MIN, P_WAYPOINT_DISTANCE_MAX = 0, 75
P_NUM_WAYPOINTS = 5
P_REACH_REWARD = 1
P_AC_SPD = 150
P_D_HEADING = 45


def plan_obs_sizes():
    return {k: P_NUM_WAYPOINTS for k in PLAN_OBS_KEYS}


def flatten_obs(obs: dict, keys) -> np.ndarray:
    return np.concatenate([np.asarray(obs[k], np.float64).reshape(obs[k].shape[0], -1)
                           for k in keys], axis=1)


# =======================================================================================
class _Base:
    kind = None
    # descent_env.py:162-182 / plan_waypoint_env.py:156-171: reset() does not clear the
    # traffic, so after a truncation (the aircraft is only deleted on termination,
    # descent_env.py:201-204, plan_waypoint_env.py:189-193) cre('KL001') is refused and the
    # next episode continues with the old aircraft.  ``present`` tracks that aircraft.
    keeps_aircraft = False
    route_lat = np.zeros(0)
    route_lon = np.zeros(0)
    route_next_qdr = np.zeros(0)

    def __init__(self, num_envs, num_ac, action_frequency, simdt, max_episode_steps,
                 autoreset=AUTORESET_NEXT_STEP, seed=0):
        self.E = int(num_envs)
        self.N = int(num_ac)
        self.S = int(action_frequency)
        self.dt = float(simdt)
        self.max_steps = int(max_episode_steps)
        self.autoreset = autoreset
        self.seed = int(seed)
        self.st = bsx.TrafState((self.E, self.N))
        self.step_count = np.zeros(self.E, np.int32)
        self.episode = np.zeros(self.E, np.int64)
        self.needs_reset = np.zeros(self.E, bool)
        self.total_reward = np.zeros(self.E, np.float64)
        self.total_intrusions = np.zeros(self.E, np.int32)
        self.env_ids = np.arange(self.E)     # global env ids (Philox counter word 0)
        self.present = np.zeros(self.E, bool)  # keeps_aircraft kinds: KL001 exists
        self.wind = None                     # bsx.WindField (wrappers/wind.py) or None
        self.wind_augment = False

    def set_wind(self, field, augment_obs=False):
        """WindFieldWrapper (bluesky_gym/wrappers/wind.py:8-24): a wind field applied to
        every env; augment_obs adds the wind_u / wind_v observation keys."""
        if self.wind_augment != bool(augment_obs):
            self.obs_dim += 2 if augment_obs else -2
        self.wind = field
        self.wind_augment = bool(augment_obs)

    def _flat(self, obs, keys):
        if self.wind_augment:
            wu, wv = bsx.wind_obs(self.st, self.wind)
            obs["wind_u"] = wu[:, None]
            obs["wind_v"] = wv[:, None]
            keys = tuple(sorted(tuple(keys) + ("wind_u", "wind_v")))
        return flatten_obs(obs, keys)

    # -------- spawn parameters (host-supplied = parity mode; None = device Philox) -----
    def device_spawn_params(self, env_ids, episodes):
        raise NotImplementedError

    def reset(self, env_mask=None, spawn=None):
        """Reset the envs in env_mask with spawn parameters (rows indexed by env id;
        None -> the device Philox draw for (seed, env, episode))."""
        mask = np.ones(self.E, bool) if env_mask is None else np.asarray(env_mask, bool)
        ids = np.nonzero(mask)[0]
        if len(ids) == 0:
            return self.observe()
        if spawn is None:
            spawn = np.zeros((self.E, self.spawn_width()), np.float64)
            spawn[ids] = self.device_spawn_params(self.env_ids[ids], self.episode[ids])
        self._reset_ids(ids, np.asarray(spawn, np.float64))
        self.present[ids] = True
        self.episode[ids] += 1          # every reset consumes one Philox episode counter
        self.step_count[ids] = 0
        self.needs_reset[ids] = False
        self.total_reward[ids] = 0.0
        self.total_intrusions[ids] = 0
        return self.observe()

    def _substeps(self):
        for _ in range(self.S):
            bsx.traffic_update(self.st, self.dt, self.route_lat, self.route_lon,
                               self.route_next_qdr, self.wind)

    def step(self, actions, spawn=None):
        """Vector step.  Returns dict: obs (flat f64), reward, terminated, truncated,
        final_obs (SAME_STEP only), was_reset, plus kind-specific diagnostics."""
        actions = np.asarray(actions, np.float64).reshape(self.E, -1)
        was_reset = self.needs_reset.copy() if self.autoreset == AUTORESET_NEXT_STEP \
            else np.zeros(self.E, bool)
        live = ~was_reset
        # snapshot of the NEXT_STEP resets: done first, then stepped envs are frozen
        pre = self.st.copy()
        self._apply_action(actions)
        self._substeps()
        res = self._observe_and_reward()
        # frozen (resetting) envs keep their pre-state; they get reset below
        for f in bsx.FIELDS_F64:
            getattr(self.st, f)[was_reset] = getattr(pre, f)[was_reset]
        self.st.swlnav[was_reset] = pre.swlnav[was_reset]
        self.st.actwp[was_reset] = pre.actwp[was_reset]
        self._commit(res, live)
        self.step_count[live] += 1
        term = res["terminated"] & live
        if self.keeps_aircraft:
            self.present[term] = False      # the terminal step deletes the aircraft
        trunc = (self.step_count >= self.max_steps) & live if self.max_steps > 0 \
            else np.zeros(self.E, bool)
        if "truncated_env" in res:          # SectorCR: ownship left the sector
            trunc = trunc | (res["truncated_env"] & live)
        reward = np.where(live, res["reward"], 0.0)
        obs = res["obs"].copy()
        done = term | trunc
        final_obs = None
        if was_reset.any():
            ro = self.reset(was_reset, spawn)
            obs[was_reset] = ro["obs"][was_reset]
            if "cd" in res:
                # a NEXT_STEP reset step reports conflict detection on the fresh state
                self._cd_into(res, was_reset)
            # ... and the reset observation's top-K (merge_env.py:124 -> _get_obs's argsort,
            # :196); no intrusion check runs at a reset (merge_env.py:103-130), so its mask is 0
            if "topk" in ro and "topk" in res:
                res["topk"] = np.where(was_reset[:, None], ro["topk"], res["topk"])
            if "intr_mask" in res:
                res["intr_mask"] = np.where(was_reset, np.uint64(0), res["intr_mask"]).astype(np.uint64)
        if self.autoreset == AUTORESET_NEXT_STEP:
            self.needs_reset = done.copy()
        elif self.autoreset == AUTORESET_SAME_STEP and done.any():
            final_obs = obs.copy()
            ro = self.reset(done, spawn)
            obs[done] = ro["obs"][done]
        out = dict(res)
        out.update(obs=obs, reward=reward, terminated=term, truncated=trunc,
                   final_obs=final_obs, was_reset=was_reset)
        return out


# =======================================================================================
class MergeOracle(_Base):
    """MergeEnv-v0 (merge_env.py).  Aircraft 0 = KL001 (ownship), 1..N-1 = INT{i-1}."""
    kind = "merge"
    route_lat = np.array([FIX_LAT, RWY_LAT])
    route_lon = np.array([FIX_LON, RWY_LON])
    route_next_qdr = np.array([float(bsx.qdrdist(FIX_LAT, FIX_LON, RWY_LAT, RWY_LON)[0]), -999.0])

    def __init__(self, num_envs, num_ac=20, num_ac_state=5, action_frequency=10, simdt=5.0,
                 max_episode_steps=50, autoreset=AUTORESET_NEXT_STEP, seed=0,
                 compute_cd=True, ac_spd=MERGE_AC_SPD, params=None):
        """ac_spd: creation CAS of every aircraft (merge_env.py:30 AC_SPD = 100; another value
        restates the logged revision of DESIGN.md §5, tests/test_ref_logs.py).  params:
        {name: value} overriding merge_env.py:13-28's module constants by their names
        (D_HEADING, D_SPEED, INTRUSION_DISTANCE, DISTANCE_MARGIN, REACH_REWARD, DRIFT_PENALTY,
        INTRUSION_PENALTY, SPAWN_DISTANCE_MIN/MAX, INTRUDER_DISTANCE_MIN/MAX), as a caller
        patching the reference module would."""
        super().__init__(num_envs, num_ac, action_frequency, simdt, max_episode_steps,
                         autoreset, seed)
        assert num_ac - 1 >= num_ac_state
        self.ac_spd = float(ac_spd)
        self.k = dict(D_HEADING=MERGE_D_HEADING, D_SPEED=MERGE_D_SPEED,
                      INTRUSION_DISTANCE=MERGE_INTRUSION_DISTANCE,
                      DISTANCE_MARGIN=MERGE_DISTANCE_MARGIN, REACH_REWARD=MERGE_REACH_REWARD,
                      DRIFT_PENALTY=MERGE_DRIFT_PENALTY, INTRUSION_PENALTY=MERGE_INTRUSION_PENALTY,
                      SPAWN_DISTANCE_MIN=MERGE_SPAWN_DISTANCE_MIN,
                      SPAWN_DISTANCE_MAX=MERGE_SPAWN_DISTANCE_MAX,
                      INTRUDER_DISTANCE_MIN=MERGE_INTRUDER_DISTANCE_MIN,
                      INTRUDER_DISTANCE_MAX=MERGE_INTRUDER_DISTANCE_MAX)
        unknown = set(params or {}) - set(self.k)
        assert not unknown, f"unknown Merge constants {sorted(unknown)}"
        self.k.update(params or {})
        self.K = int(num_ac_state)
        self.compute_cd = compute_cd
        self.wpt_reach = np.zeros(self.E, np.int32)
        self.faf_reached = np.zeros(self.E, np.int32)
        self.drift_sum = np.zeros(self.E, np.float64)
        self.drift_cnt = np.zeros(self.E, np.int32)
        self.obs_sizes = merge_obs_sizes(self.K)
        self.obs_dim = sum(self.obs_sizes.values())

    def spawn_width(self):
        return 2 * self.N

    def device_spawn_params(self, env_ids, episodes):
        j = np.arange(self.N, dtype=np.uint32)[None, :]
        x0, x1, x2, x3 = philox.philox4x32_10(np.asarray(env_ids, np.uint32)[:, None],
                                              np.asarray(episodes, np.uint32)[:, None],
                                              j, philox.TAG_MERGE, self.seed)
        ua = philox.u01_53(x0, x1)
        ub = philox.u01_53(x2, x3)
        k = self.k
        a, b = -k["D_HEADING"], k["D_HEADING"]
        brg = a + (b - a) * ua
        dmin = np.where(j == 0, k["SPAWN_DISTANCE_MIN"], k["INTRUDER_DISTANCE_MIN"]).astype(np.float64)
        dmax = np.where(j == 0, k["SPAWN_DISTANCE_MAX"], k["INTRUDER_DISTANCE_MAX"]).astype(np.float64)
        dist = dmin + (dmax - dmin) * ub
        out = np.empty((len(env_ids), 2 * self.N))
        out[:, 0::2] = brg
        out[:, 1::2] = dist
        return out

    def _reset_ids(self, ids, spawn):
        """merge_env.py:103-130 + _gen_aircraft :148-158."""
        st = self.st
        brg = spawn[ids][:, 0::2]
        dist = spawn[ids][:, 1::2]
        lat, lon = bsx.get_point_at_distance(FIX_LAT, FIX_LON, dist, brg)
        for j in range(self.N):
            bsx.cre_state(st, (ids, np.full(len(ids), j)), lat[:, j], lon[:, j],
                          brg[:, j] - 180, MERGE_ALT, self.ac_spd)
        # intruders: ADDWPT FIX ; DEST RWY  -> LNAV on, active waypoint FIX
        st.swlnav[ids, 1:] = True
        st.actwp[ids, 1:] = 0
        self.wpt_reach[ids] = 0
        self.faf_reached[ids] = 0
        self.drift_sum[ids] = 0.0
        self.drift_cnt[ids] = 0

    def _apply_action(self, actions):
        """merge_env.py:286-293 + BlueSky HDG / SPD stack commands."""
        st = self.st
        dh = actions[:, 0] * self.k["D_HEADING"]
        dv = actions[:, 1] * self.k["D_SPEED"]
        heading_new = bsx.bound_angle_positive_negative_180(st.hdg[:, 0] + dh)
        speed_new = (st.cas[:, 0] + dv) * MPS2KT
        st.ap_trk[:, 0] = bsx.selhdg_track(st, (slice(None), 0), heading_new, self.wind)
        st.swlnav[:, 0] = False
        st.selspd[:, 0] = np.where(speed_new >= 1.0, speed_new * bsx.kts, speed_new)

    def _obs_core(self):
        """merge_env.py:160-236 (_get_obs)."""
        st = self.st
        E, N, K = self.E, self.N, self.K
        lat0, lon0 = st.lat[:, 0], st.lon[:, 0]
        hdg0, tas0 = st.hdg[:, 0], st.tas[:, 0]
        wlat = np.where(self.wpt_reach == 0, FIX_LAT, RWY_LAT)
        wlon = np.where(self.wpt_reach == 0, FIX_LON, RWY_LON)
        wpt_qdr, wpt_dist = bsx.kwikqdrdist(lat0, lon0, wlat, wlon)
        drift = bsx.bound_angle_positive_negative_180(hdg0 - wpt_qdr)
        cos_drift = np.cos(np.deg2rad(drift))
        sin_drift = np.sin(np.deg2rad(drift))
        vx = np.cos(np.deg2rad(hdg0)) * tas0
        vy = np.sin(np.deg2rad(hdg0)) * tas0
        distances = bsx.kwikdist_matrix(lat0[:, None], lon0[:, None], st.lat[:, 1:], st.lon[:, 1:])
        order = np.argsort(distances, axis=1, kind="stable")
        brg, dist = bsx.kwikqdrdist(lat0[:, None], lon0[:, None], st.lat[:, 1:], st.lon[:, 1:])
        x_r = (dist * NM2KM * 1000) * np.cos(np.deg2rad(brg))
        y_r = (dist * NM2KM * 1000) * np.sin(np.deg2rad(brg))
        vx_int = np.cos(np.deg2rad(st.hdg[:, 1:])) * st.tas[:, 1:]
        vy_int = np.sin(np.deg2rad(st.hdg[:, 1:])) * st.tas[:, 1:]
        vx_r = vx_int - vx[:, None]
        vy_r = vy_int - vy[:, None]
        track = np.arctan2(vy_r, vx_r)
        top = order[:, :K]
        take = lambda a: np.take_along_axis(a, top, axis=1)
        obs = {
            "cos(drift)": cos_drift[:, None],
            "sin(drift)": sin_drift[:, None],
            "airspeed": tas0[:, None],
            "waypoint_dist": (wpt_dist / 250)[:, None],
            "faf_reached": self.wpt_reach.astype(np.float64)[:, None],
            "x_r": take(x_r) / 1000000,
            "y_r": take(y_r) / 1000000,
            "vx_r": take(vx_r) / 150,
            "vy_r": take(vy_r) / 150,
            "cos(track)": np.cos(take(track)),
            "sin(track)": np.sin(take(track)),
            "distances": take(distances) / 250,
        }
        return obs, drift, wpt_dist, dist, top + 1

    def observe(self):
        obs, _drift, _wd, _dist, topk = self._obs_core()
        return {"obs": self._flat(obs, MERGE_OBS_KEYS), "obs_dict": obs, "topk": topk}

    def _observe_and_reward(self):
        obs, drift, wpt_dist, dist, topk = self._obs_core()
        # _check_waypoint (merge_env.py:257-268)
        wr = self.wpt_reach.copy()
        faf = self.faf_reached.copy()
        k = self.k
        c1 = (wpt_dist < k["DISTANCE_MARGIN"]) & (wr != 1)
        c2 = ~c1 & (wpt_dist < 2 * k["DISTANCE_MARGIN"]) & (wr == 1)
        reach_reward = np.where(c1, k["REACH_REWARD"], 0)
        new_wr = np.where(c1, 1, wr)
        new_faf = np.where(c1, 1, np.where(c2, 2, faf))
        done = c2
        # _check_drift (:270-273)
        d = np.abs(np.deg2rad(drift))
        drift_reward = d * k["DRIFT_PENALTY"]
        # _check_intrusion (:275-284), intruders by index
        intr = dist < k["INTRUSION_DISTANCE"]
        nintr = intr.sum(axis=1)
        intrusion_reward = nintr * k["INTRUSION_PENALTY"]
        reward = reach_reward + drift_reward + intrusion_reward
        intr_mask = np.zeros(self.E, np.uint64)
        for i in range(self.N - 1):
            intr_mask |= intr[:, i].astype(np.uint64) << np.uint64(i + 1)
        res = dict(obs=self._flat(obs, MERGE_OBS_KEYS), obs_dict=obs, reward=reward,
                   terminated=done, topk=topk, intr_mask=intr_mask, nintr=nintr,
                   _new_wr=new_wr, _new_faf=new_faf, _d=d)
        if self.compute_cd:
            cd = bsx.statebased_detect(self.st.lat, self.st.lon, self.st.alt, self.st.trk,
                                       self.st.gs, self.st.vs)
            res["conf_mask"] = _rows_to_u64(cd["swconfl"])
            res["los_mask"] = _rows_to_u64(cd["swlos"])
            res["tcpamax"] = cd["tcpamax"]
            res["min_sep"] = cd["min_sep"]
            res["cd"] = cd
        return res

    def _commit(self, res, live):
        self.wpt_reach = np.where(live, res["_new_wr"], self.wpt_reach).astype(np.int32)
        self.faf_reached = np.where(live, res["_new_faf"], self.faf_reached).astype(np.int32)
        self.drift_sum = np.where(live, self.drift_sum + res["_d"], self.drift_sum)
        self.drift_cnt = self.drift_cnt + live
        self.total_intrusions = self.total_intrusions + np.where(live, res["nintr"], 0).astype(np.int32)
        self.total_reward = np.where(live, self.total_reward + res["reward"], self.total_reward)

    def info(self):
        with np.errstate(invalid="ignore", divide="ignore"):
            avg = self.drift_sum / self.drift_cnt
        return {"total_reward": self.total_reward.copy(), "faf_reach": self.faf_reached.copy(),
                "average_drift": np.where(self.drift_cnt > 0, avg, np.nan),
                "total_intrusions": self.total_intrusions.copy()}


# =======================================================================================
class _VertBase(_Base):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.target_alt = np.zeros(self.E, np.float64)
        self.final_altitude = np.zeros(self.E, np.float64)

    def _apply_action(self, actions):
        """vertical_cr_env.py:242-256 / descent_env.py:146-160."""
        a = actions[:, 0] * ACTION_2_MS
        st = self.st
        up = a >= 0
        dn = a < 0
        st.selalt[:, 0] = np.where(up, 1000000.0, np.where(dn, 0.0, st.selalt[:, 0]))
        st.selvs[:, 0] = np.where(up | dn, a, st.selvs[:, 0])

    def _own_reset(self, ids, spawn):
        self.target_alt[ids] = spawn[ids, 1]
        self.final_altitude[ids] = 0.0
        if self.keeps_aircraft:
            ids = ids[~self.present[ids]]   # cre('KL001') refused: aircraft kept
        alt_init = spawn[ids, 0]
        st = self.st
        for j in range(self.N):
            bsx.cre_state(st, (ids, np.full(len(ids), j)), 0.0, 0.0, 0.0, 0.0, 0.0)
        # cre('KL001', acalt=alt_init, acspd=150) with default aclat=52, aclon=4, achdg=0
        bsx.cre_state(st, (ids, np.zeros(len(ids), int)), 52.0, 4.0, 0.0, alt_init, V_AC_SPD)

    def _alt_reward(self, altitude, runway_distance):
        """vertical_cr_env.py:216-225 / descent_env.py:131-144."""
        c1 = (runway_distance > 0) & (altitude > 0)
        c2 = ~c1 & (altitude <= 0)
        c3 = ~c1 & ~c2 & (runway_distance <= 0)
        alt_pen = np.where(c1, np.abs(self.target_alt - altitude) * V_ALT_DIF_REWARD_SCALE,
                           np.where(c2, V_CRASH_PENALTY, altitude * V_RWY_ALT_DIF_REWARD_SCALE))
        fin = np.where(c2, -100.0, np.where(c3, altitude, self.final_altitude))
        return alt_pen, c2 | c3, fin

    @staticmethod
    def _randint_int_bounds(alt_init):
        return alt_init


class VerticalOracle(_VertBase):
    """VerticalCREnv-v0 (vertical_cr_env.py).  N = 1 + NUM_INTRUDERS."""
    kind = "vertical"

    def __init__(self, num_envs, num_ac=6, action_frequency=30, simdt=1.0,
                 max_episode_steps=300, autoreset=AUTORESET_NEXT_STEP, seed=0,
                 compute_cd=True):
        super().__init__(num_envs, num_ac, action_frequency, simdt, max_episode_steps,
                         autoreset, seed)
        self.NI = self.N - 1
        self.compute_cd = compute_cd
        self.obs_sizes = vertical_obs_sizes(self.NI)
        self.obs_dim = sum(self.obs_sizes.values())

    def spawn_width(self):
        return 2 + 4 * self.NI

    def device_spawn_params(self, env_ids, episodes):
        ids = np.asarray(env_ids, np.uint32)
        eps = np.asarray(episodes, np.uint32)
        x0, x1, _, _ = philox.philox4x32_10(ids, eps, 0, philox.TAG_VERT, self.seed)
        alt_init = philox.randint_u32(x0, ALT_MIN, ALT_MAX)
        target = alt_init + philox.randint_u32(x1, -TARGET_ALT_DIF, TARGET_ALT_DIF)
        out = np.zeros((len(ids), self.spawn_width()))
        out[:, 0] = alt_init
        out[:, 1] = target
        spd = bsx.vcas2tas(np.float64(V_AC_SPD), alt_init.astype(np.float64))
        for i in range(self.NI):
            y0, y1, y2, y3 = philox.philox4x32_10(ids, eps, i + 1, philox.TAG_VERT, self.seed)
            params = vertical_conflict_ints(alt_init.astype(np.float64), target.astype(np.float64),
                                            spd, y0, y1, y2, y3)
            out[:, 2 + 4 * i: 6 + 4 * i] = np.stack(params, axis=1)
        return out

    def _reset_ids(self, ids, spawn):
        """vertical_cr_env.py:258-281 + _generate_conflicts :183-200 (creconfs)."""
        self._own_reset(ids, spawn)
        st = self.st
        for e in ids:
            alt0 = float(st.alt[e, 0])
            gs0 = float(st.tas[e, 0])
            for i in range(self.NI):
                dpsi, cpa, tlosh, dH = spawn[e, 2 + 4 * i: 6 + 4 * i]
                lat, lon, hdg, acalt, acspd, acvs = bsx.creconfs_params(
                    52.0, 4.0, alt0, 0.0, gs0, 0.0, float(dpsi), float(cpa), float(tlosh),
                    dH=float(dH), tlosv=100000000000.0)
                bsx.cre_state(st, (e, i + 1), lat, lon, hdg, acalt, acspd)
                st.vs[e, i + 1] = acvs
                # traf.alt[i+1] = alt[target] + dH ; ap.selaltcmd(i+1, alt[target] + dH, 0)
                st.alt[e, i + 1] = alt0 + dH
                st.selalt[e, i + 1] = alt0 + dH
                st.selvs[e, i + 1] = acvs   # selaltcmd(..., vspd=acvs) from creconfs; 0 keeps it

    def _obs_core(self):
        """vertical_cr_env.py:113-181."""
        st = self.st
        lat0, lon0, hdg0 = st.lat[:, :1], st.lon[:, :1], st.hdg[:, :1]
        altitude = st.alt[:, 0]
        vz = st.vs[:, 0]
        int_qdr, int_dis = bsx.kwikqdrdist(lat0, lon0, st.lat[:, 1:], st.lon[:, 1:])
        intruder_distance = int_dis * NM2KM
        alt_dif = st.alt[:, 1:] - altitude[:, None]
        vz_dif = st.vs[:, 1:] - vz[:, None]
        bearing = bsx.bound_angle_positive_negative_180(hdg0 - int_qdr)
        cosb = np.cos(np.deg2rad(bearing))
        sinb = np.sin(np.deg2rad(bearing))
        hd = hdg0 - st.hdg[:, 1:]
        x_dif = -np.cos(np.deg2rad(hd)) * st.gs[:, 1:]
        y_dif = st.gs[:, :1] - np.sin(np.deg2rad(hd)) * st.gs[:, 1:]
        runway_distance = DEFAULT_RWY_DIS - bsx.kwikdist(V_RWY_LAT, V_RWY_LON, st.lat[:, 0], st.lon[:, 0]) * NM2KM
        obs = {
            "altitude": ((altitude - ALT_MEAN) / ALT_STD)[:, None],
            "vz": ((vz - VZ_MEAN) / VZ_STD)[:, None],
            "target_altitude": ((self.target_alt - ALT_MEAN) / ALT_STD)[:, None],
            "runway_distance": ((runway_distance - RWY_DIS_MEAN) / RWY_DIS_STD)[:, None],
            "intruder_distance": intruder_distance / DEFAULT_RWY_DIS,
            "cos_difference_pos": cosb,
            "sin_difference_pos": sinb,
            "altitude_difference": alt_dif / ALT_STD,
            "x_difference_speed": x_dif / V_AC_SPD,
            "y_difference_speed": y_dif / V_AC_SPD,
            "z_difference_speed": vz_dif,
        }
        return obs, altitude, runway_distance, int_dis

    def observe(self):
        obs, *_ = self._obs_core()
        return {"obs": self._flat(obs, VERTICAL_OBS_KEYS), "obs_dict": obs}

    def _observe_and_reward(self):
        obs, altitude, runway_distance, int_dis = self._obs_core()
        st = self.st
        vert_dis = st.alt[:, :1] - st.alt[:, 1:]
        intr = (int_dis < V_INTRUSION_DISTANCE) & (np.abs(vert_dis) < V_VERTICAL_MARGIN)
        nintr = intr.sum(axis=1)
        int_penalty = nintr * V_INTRUSION_PENALTY
        alt_pen, done, fin = self._alt_reward(altitude, runway_distance)
        reward = alt_pen + int_penalty
        intr_mask = np.zeros(self.E, np.uint64)
        for i in range(self.NI):
            intr_mask |= intr[:, i].astype(np.uint64) << np.uint64(i + 1)
        res = dict(obs=self._flat(obs, VERTICAL_OBS_KEYS), obs_dict=obs, reward=reward,
                   terminated=done, intr_mask=intr_mask, nintr=nintr, _fin=fin)
        if self.compute_cd:
            cd = bsx.statebased_detect(st.lat, st.lon, st.alt, st.trk, st.gs, st.vs)
            res["conf_mask"] = _rows_to_u64(cd["swconfl"])
            res["los_mask"] = _rows_to_u64(cd["swlos"])
            res["tcpamax"] = cd["tcpamax"]
            res["min_sep"] = cd["min_sep"]
            res["cd"] = cd
        return res

    def _commit(self, res, live):
        self.final_altitude = np.where(live, res["_fin"], self.final_altitude)
        self.total_intrusions = self.total_intrusions + np.where(live, res["nintr"], 0).astype(np.int32)
        self.total_reward = np.where(live, self.total_reward + res["reward"], self.total_reward)

    def info(self):
        return {"total_reward": self.total_reward.copy(),
                "total_intrusions": self.total_intrusions.copy(),
                "final_altitude": self.final_altitude.copy()}


def vertical_conflict_ints(altitude, target_alt, spd, y0, y1, y2, y3):
    """Device-mode draw of (dpsi, cpa, tlosh, dH) following the distributions of
    vertical_cr_env.py:187-195 with Philox uint32 draws (multiply-shift randint)."""
    dpsi = philox.randint_u32(y0, 45, 315)
    cpa = philox.randint_u32(y1, 0, V_INTRUSION_DISTANCE_INT)
    hi_t = np.trunc(((DEFAULT_RWY_DIS * 0.9) * 1000) / spd).astype(np.int64)
    tlosh = philox.randint_u32(y2, 100, hi_t)
    average_tod = (DEFAULT_RWY_DIS * 1000 / spd) - 2 * target_alt / ACTION_2_MS
    lo_a = np.trunc(-altitude + 500).astype(np.int64)
    hi_a = np.trunc((target_alt - altitude) + 100).astype(np.int64)
    lo_b = np.trunc((target_alt - altitude) - 500).astype(np.int64)
    hi_b = np.trunc((target_alt - altitude) + 500).astype(np.int64)
    late = tlosh > average_tod
    dH = philox.randint_u32(y3, np.where(late, lo_a, lo_b), np.where(late, hi_a, hi_b))
    return (dpsi.astype(np.float64), cpa.astype(np.float64), tlosh.astype(np.float64),
            dH.astype(np.float64))


class DescentOracle(_VertBase):
    """DescentEnv-v0 (descent_env.py).  N = 1."""
    kind = "descent"
    keeps_aircraft = True

    def __init__(self, num_envs, action_frequency=30, simdt=1.0, max_episode_steps=300,
                 autoreset=AUTORESET_NEXT_STEP, seed=0):
        super().__init__(num_envs, 1, action_frequency, simdt, max_episode_steps,
                         autoreset, seed)
        self.obs_sizes = descent_obs_sizes()
        self.obs_dim = 4

    def spawn_width(self):
        return 2

    def device_spawn_params(self, env_ids, episodes):
        x0, x1, _, _ = philox.philox4x32_10(np.asarray(env_ids, np.uint32),
                                            np.asarray(episodes, np.uint32), 0,
                                            philox.TAG_DESC, self.seed)
        alt_init = philox.randint_u32(x0, ALT_MIN, ALT_MAX)
        target = alt_init + philox.randint_u32(x1, -TARGET_ALT_DIF, TARGET_ALT_DIF)
        return np.stack([alt_init, target], axis=1).astype(np.float64)

    def _reset_ids(self, ids, spawn):
        """descent_env.py:162-182."""
        self._own_reset(ids, spawn)

    def _obs_core(self):
        """descent_env.py:89-117."""
        st = self.st
        altitude = st.alt[:, 0]
        vz = st.vs[:, 0]
        runway_distance = DEFAULT_RWY_DIS - bsx.kwikdist(V_RWY_LAT, V_RWY_LON, st.lat[:, 0], st.lon[:, 0]) * NM2KM
        obs = {
            "altitude": ((altitude - ALT_MEAN) / ALT_STD)[:, None],
            "vz": ((vz - VZ_MEAN) / VZ_STD)[:, None],
            "target_altitude": ((self.target_alt - ALT_MEAN) / ALT_STD)[:, None],
            "runway_distance": ((runway_distance - RWY_DIS_MEAN) / RWY_DIS_STD)[:, None],
        }
        return obs, altitude, runway_distance

    def observe(self):
        obs, *_ = self._obs_core()
        return {"obs": self._flat(obs, DESCENT_OBS_KEYS), "obs_dict": obs}

    def _observe_and_reward(self):
        obs, altitude, runway_distance = self._obs_core()
        alt_pen, done, fin = self._alt_reward(altitude, runway_distance)
        return dict(obs=self._flat(obs, DESCENT_OBS_KEYS), obs_dict=obs, reward=alt_pen,
                    terminated=done, _fin=fin)

    def _commit(self, res, live):
        self.final_altitude = np.where(live, res["_fin"], self.final_altitude)
        self.total_reward = np.where(live, self.total_reward + res["reward"], self.total_reward)

    def info(self):
        return {"total_reward": self.total_reward.copy(),
                "final_altitude": self.final_altitude.copy()}


def _cd_fill(o, res, mask):
    st = o.st
    cd = bsx.statebased_detect(st.lat, st.lon, st.alt, st.trk, st.gs, st.vs)
    res["conf_mask"] = np.where(mask[:, None], _rows_to_u64(cd["swconfl"]), res["conf_mask"])
    res["los_mask"] = np.where(mask[:, None], _rows_to_u64(cd["swlos"]), res["los_mask"])
    res["tcpamax"] = np.where(mask[:, None], cd["tcpamax"], res["tcpamax"])
    res["min_sep"] = np.where(mask, cd["min_sep"], res["min_sep"])


_Base._cd_into = lambda self, res, mask: _cd_fill(self, res, mask)


class HorizontalOracle(_Base):
    """HorizontalCREnv-v0 (horizontal_cr_env.py).  N = 1 + NUM_INTRUDERS."""
    kind = "horizontal"

    def __init__(self, num_envs, num_ac=6, action_frequency=10, simdt=5.0,
                 max_episode_steps=300, autoreset=AUTORESET_NEXT_STEP, seed=0,
                 compute_cd=True):
        super().__init__(num_envs, num_ac, action_frequency, simdt, max_episode_steps,
                         autoreset, seed)
        self.NI = self.N - 1
        self.compute_cd = compute_cd
        self.obs_sizes = horizontal_obs_sizes(self.NI)
        self.obs_dim = sum(self.obs_sizes.values())
        self.wpt_lat = np.zeros(self.E)
        self.wpt_lon = np.zeros(self.E)
        self.wpt_reach = np.zeros(self.E, np.int32)
        self.drift_sum = np.zeros(self.E)
        self.drift_cnt = np.zeros(self.E, np.int32)

    def spawn_width(self):
        return 3 * self.NI + 1

    def device_spawn_params(self, env_ids, episodes):
        ids = np.asarray(env_ids, np.uint32)
        eps = np.asarray(episodes, np.uint32)
        out = np.zeros((len(ids), self.spawn_width()))
        for i in range(self.NI):
            y0, y1, y2, _ = philox.philox4x32_10(ids, eps, i + 1, philox.TAG_HORZ, self.seed)
            out[:, 3 * i] = philox.randint_u32(y0, 45, 315)
            out[:, 3 * i + 1] = philox.randint_u32(y1, 0, H_INTRUSION_DISTANCE)
            out[:, 3 * i + 2] = philox.randint_u32(y2, 100, 1000)
        x0, _, _, _ = philox.philox4x32_10(ids, eps, 0, philox.TAG_HORZ, self.seed)
        out[:, -1] = philox.randint_u32(x0, H_WAYPOINT_DISTANCE_MIN, H_WAYPOINT_DISTANCE_MAX)
        return out

    def _reset_ids(self, ids, spawn):
        """horizontal_cr_env.py:82-101 + _generate_conflicts :127-133 + _generate_waypoint
        :135-148."""
        st = self.st
        for j in range(self.N):
            bsx.cre_state(st, (ids, np.full(len(ids), j)), 0.0, 0.0, 0.0, 0.0, 0.0)
        # cre('KL001', acspd=150): default 52N 4E, hdg 0, alt 0
        bsx.cre_state(st, (ids, np.zeros(len(ids), int)), 52.0, 4.0, 0.0, 0.0, H_AC_SPD)
        for e in ids:
            gs0 = float(st.tas[e, 0])
            for i in range(self.NI):
                dpsi, cpa, tlosh = spawn[e, 3 * i: 3 * i + 3]
                lat, lon, hdg, acalt, acspd, acvs = bsx.creconfs_params(
                    52.0, 4.0, 0.0, 0.0, gs0, 0.0, float(dpsi), float(cpa), float(tlosh))
                bsx.cre_state(st, (e, i + 1), lat, lon, hdg, acalt, acspd)
                st.vs[e, i + 1] = acvs
                st.selalt[e, i + 1] = 0.0
            wlat, wlon = bsx.get_point_at_distance(st.lat[e, 0], st.lon[e, 0], spawn[e, -1], 0)
            self.wpt_lat[e], self.wpt_lon[e] = float(wlat), float(wlon)
        self.wpt_reach[ids] = 0
        self.drift_sum[ids] = 0.0
        self.drift_cnt[ids] = 0

    def _apply_action(self, actions):
        """horizontal_cr_env.py:272-275: HDG = hdg + a*45 (no wrap), LNAV off."""
        st = self.st
        st.ap_trk[:, 0] = bsx.selhdg_track(st, (slice(None), 0),
                                           st.hdg[:, 0] + actions[:, 0] * H_D_HEADING, self.wind)
        st.swlnav[:, 0] = False

    def _obs_core(self):
        """horizontal_cr_env.py:150-213."""
        st = self.st
        lat0, lon0, hdg0 = st.lat[:, :1], st.lon[:, :1], st.hdg[:, :1]
        int_qdr, int_dis = bsx.kwikqdrdist(lat0, lon0, st.lat[:, 1:], st.lon[:, 1:])
        bearing = bsx.bound_angle_positive_negative_180(hdg0 - int_qdr)
        hd = hdg0 - st.hdg[:, 1:]
        x_dif = -np.cos(np.deg2rad(hd)) * st.gs[:, 1:]
        y_dif = st.gs[:, :1] - np.sin(np.deg2rad(hd)) * st.gs[:, 1:]
        wpt_qdr, wpt_dis = bsx.kwikqdrdist(st.lat[:, 0], st.lon[:, 0], self.wpt_lat, self.wpt_lon)
        drift = bsx.bound_angle_positive_negative_180(st.hdg[:, 0] - wpt_qdr)
        obs = {
            "intruder_distance": (int_dis * NM2KM) / H_WAYPOINT_DISTANCE_MAX,
            "cos_difference_pos": np.cos(np.deg2rad(bearing)),
            "sin_difference_pos": np.sin(np.deg2rad(bearing)),
            "x_difference_speed": x_dif / H_AC_SPD,
            "y_difference_speed": y_dif / H_AC_SPD,
            "waypoint_distance": ((wpt_dis * NM2KM) / H_WAYPOINT_DISTANCE_MAX)[:, None],
            "cos_drift": np.cos(np.deg2rad(drift))[:, None],
            "sin_drift": np.sin(np.deg2rad(drift))[:, None],
        }
        return obs, int_dis, wpt_dis * NM2KM, drift

    def observe(self):
        obs, *_ = self._obs_core()
        return {"obs": self._flat(obs, HORIZONTAL_OBS_KEYS), "obs_dict": obs}

    def _observe_and_reward(self):
        obs, int_dis, wpt_km, drift = self._obs_core()
        c = (wpt_km < H_DISTANCE_MARGIN) & (self.wpt_reach != 1)
        reach = np.where(c, H_REACH_REWARD, 0)
        new_wr = np.where(c, 1, self.wpt_reach)
        d = np.abs(np.deg2rad(drift))
        intr = int_dis < H_INTRUSION_DISTANCE
        nintr = intr.sum(axis=1)
        reward = reach + d * H_DRIFT_PENALTY + nintr * H_INTRUSION_PENALTY
        intr_mask = np.zeros(self.E, np.uint64)
        for i in range(self.NI):
            intr_mask |= intr[:, i].astype(np.uint64) << np.uint64(i + 1)
        res = dict(obs=self._flat(obs, HORIZONTAL_OBS_KEYS), obs_dict=obs, reward=reward,
                   terminated=new_wr == 1, intr_mask=intr_mask, nintr=nintr, _new_wr=new_wr, _d=d)
        if self.compute_cd:
            st = self.st
            cd = bsx.statebased_detect(st.lat, st.lon, st.alt, st.trk, st.gs, st.vs)
            res["conf_mask"] = _rows_to_u64(cd["swconfl"])
            res["los_mask"] = _rows_to_u64(cd["swlos"])
            res["tcpamax"] = cd["tcpamax"]
            res["min_sep"] = cd["min_sep"]
            res["cd"] = cd
        return res

    def _commit(self, res, live):
        self.wpt_reach = np.where(live, res["_new_wr"], self.wpt_reach).astype(np.int32)
        self.drift_sum = np.where(live, self.drift_sum + res["_d"], self.drift_sum)
        self.drift_cnt = self.drift_cnt + live
        self.total_intrusions = self.total_intrusions + np.where(live, res["nintr"], 0).astype(np.int32)
        self.total_reward = np.where(live, self.total_reward + res["reward"], self.total_reward)

    def info(self):
        with np.errstate(invalid="ignore", divide="ignore"):
            avg = self.drift_sum / self.drift_cnt
        return {"total_reward": self.total_reward.copy(),
                "total_intrusions": self.total_intrusions.copy(),
                "average_drift": np.where(self.drift_cnt > 0, avg, np.nan)}


def horizontal_spawn_from_np_random(rs, num_intruders):
    """np.random draws of horizontal_cr_env.py:130-132 (per intruder) then :140."""
    out = []
    for _ in range(num_intruders):
        out += [float(rs.randint(45, 315)), float(rs.randint(0, H_INTRUSION_DISTANCE)),
                float(rs.randint(100, 1000))]
    out.append(float(rs.randint(H_WAYPOINT_DISTANCE_MIN, H_WAYPOINT_DISTANCE_MAX)))
    return np.array(out, np.float64)


def _rows_to_u64(m):
    """bool [..., N, N] -> uint64 [..., N] with bit j of row i = m[i, j] (N <= 64)."""
    n = m.shape[-1]
    w = (np.uint64(1) << np.arange(n, dtype=np.uint64))
    return (m.astype(np.uint64) * w).sum(axis=-1, dtype=np.uint64)


def merge_spawn_from_python_random(rng, num_ac):
    """The 2 + 2*(N-1) random.uniform draws of merge_env.py:115-116,150-151, in order."""
    out = []
    out.append(rng.uniform(-MERGE_D_HEADING, MERGE_D_HEADING))
    out.append(rng.uniform(MERGE_SPAWN_DISTANCE_MIN, MERGE_SPAWN_DISTANCE_MAX))
    for _ in range(num_ac - 1):
        out.append(rng.uniform(-MERGE_D_HEADING, MERGE_D_HEADING))
        out.append(rng.uniform(MERGE_INTRUDER_DISTANCE_MIN, MERGE_INTRUDER_DISTANCE_MAX))
    return np.array(out, np.float64)


def vertical_spawn_from_np_random(rs, num_intruders, compute_spd):
    """The legacy np.random draws of vertical_cr_env.py:267-268,187-195, in order.
    compute_spd(alt_init) -> ownship ground speed after cre (tas)."""
    alt_init = rs.randint(ALT_MIN, ALT_MAX)
    target_alt = alt_init + rs.randint(-TARGET_ALT_DIF, TARGET_ALT_DIF)
    altitude = float(alt_init)
    spd = compute_spd(alt_init)
    out = [float(alt_init), float(target_alt)]
    for _ in range(num_intruders):
        dpsi = rs.randint(45, 315)
        cpa = rs.randint(0, V_INTRUSION_DISTANCE_INT)
        tlosh = rs.randint(100, int((DEFAULT_RWY_DIS * 0.9) * 1000 / spd))
        average_tod = (DEFAULT_RWY_DIS * 1000 / spd) - 2 * target_alt / ACTION_2_MS
        if tlosh > average_tod:
            dH = rs.randint(int(-altitude + 500), int((target_alt - altitude) + 100))
        else:
            dH = rs.randint(int((target_alt - altitude) - 500), int((target_alt - altitude) + 500))
        out += [float(dpsi), float(cpa), float(tlosh), float(dH)]
    return np.array(out, np.float64)


def descent_spawn_from_np_random(rs):
    alt_init = rs.randint(ALT_MIN, ALT_MAX)
    target_alt = alt_init + rs.randint(-TARGET_ALT_DIF, TARGET_ALT_DIF)
    return np.array([float(alt_init), float(target_alt)])


# =======================================================================================
class PlanWaypointOracle(_Base):
    """PlanWaypointEnv-v0 (plan_waypoint_env.py).  N = 1, five waypoints around the
    ownship's position at reset (the kept aircraft's, after a truncation)."""
    kind = "plan_waypoint"
    keeps_aircraft = True

    def __init__(self, num_envs, action_frequency=10, simdt=1.0, max_episode_steps=300,
                 autoreset=AUTORESET_NEXT_STEP, seed=0):
        super().__init__(num_envs, 1, action_frequency, simdt, max_episode_steps,
                         autoreset, seed)
        W = P_NUM_WAYPOINTS
        self.obs_sizes = plan_obs_sizes()
        self.obs_dim = 4 * W
        self.wpt_lat = np.zeros((self.E, W))
        self.wpt_lon = np.zeros((self.E, W))
        self.wpt_reach = np.zeros((self.E, W), np.int64)

    def spawn_width(self):
        return 2 * P_NUM_WAYPOINTS

    def device_spawn_params(self, env_ids, episodes):
        k = np.arange(P_NUM_WAYPOINTS, dtype=np.uint32)[None, :]
        x0, x1, _, _ = philox.philox4x32_10(np.asarray(env_ids, np.uint32)[:, None],
                                            np.asarray(episodes, np.uint32)[:, None], k,
                                            philox.TAG_PLAN, self.seed)
        dis = philox.randint_u32(x0, P_WAYPOINT_DISTANCE_MIN, P_WAYPOINT_DISTANCE_MAX)
        hdg = philox.randint_u32(x1, 0, 359)
        return np.concatenate([dis, hdg], axis=1).astype(np.float64)

    def _reset_ids(self, ids, spawn):
        """plan_waypoint_env.py:156-171 (reset) + _generate_waypoint :200-213."""
        st = self.st
        new = ids[~self.present[ids]]
        # cre('KL001', acspd=150): default 52N 4E, hdg 0, alt 0 (refused if KL001 exists)
        bsx.cre_state(st, (new, np.zeros(len(new), int)), 52.0, 4.0, 0.0, 0.0, P_AC_SPD)
        W = P_NUM_WAYPOINTS
        lat, lon = bsx.get_point_at_distance(st.lat[ids, :1], st.lon[ids, :1],
                                             spawn[ids, :W], spawn[ids, W:2 * W])
        self.wpt_lat[ids] = lat
        self.wpt_lon[ids] = lon
        self.wpt_reach[ids] = 0

    def _apply_action(self, actions):
        """plan_waypoint_env.py:148-154: HDG KL001 {hdg + a*45} (no wrap)."""
        st = self.st
        st.ap_trk[:, 0] = bsx.selhdg_track(st, (slice(None), 0),
                                           st.hdg[:, 0] + actions[:, 0] * P_D_HEADING, self.wind)
        st.swlnav[:, 0] = False

    def _obs_core(self):
        """plan_waypoint_env.py:86-124 (_get_obs), with the reach flags before _get_reward."""
        st = self.st
        qdr, dis = bsx.kwikqdrdist(st.lat[:, :1], st.lon[:, :1], self.wpt_lat, self.wpt_lon)
        dis_km = dis * NM2KM
        drift = bsx.bound_angle_positive_negative_180(st.hdg[:, :1] - qdr)
        f = (self.wpt_reach - 1) * -1          # int: 1 unreached, 0 reached
        obs = {
            "waypoint_distance": f * dis_km / P_WAYPOINT_DISTANCE_MAX,
            "cos_difference": f * np.cos(np.deg2rad(drift)),
            "sin_difference": f * np.sin(np.deg2rad(drift)),
            "waypoint_reached": self.wpt_reach.astype(np.float64),
        }
        return obs, dis_km

    def observe(self):
        obs, _ = self._obs_core()
        return {"obs": self._flat(obs, PLAN_OBS_KEYS), "obs_dict": obs}

    def _observe_and_reward(self):
        """_get_reward :135-146 + _check_waypoint :215-227."""
        obs, dis_km = self._obs_core()
        new = (dis_km < P_DISTANCE_MARGIN) & (self.wpt_reach != 1)
        reward = (new.sum(axis=1) * P_REACH_REWARD).astype(np.float64)
        new_wr = np.where(new, 1, self.wpt_reach)
        done = (new_wr == 1).all(axis=1)
        return dict(obs=self._flat(obs, PLAN_OBS_KEYS), obs_dict=obs, reward=reward,
                    terminated=done, _new_wr=new_wr)

    def _commit(self, res, live):
        self.wpt_reach = np.where(live[:, None], res["_new_wr"], self.wpt_reach)
        self.total_reward = np.where(live, self.total_reward + res["reward"], self.total_reward)

    def info(self):
        return {"total_reward": self.total_reward.copy(),
                "waypoints_completed": self.wpt_reach.sum(axis=1)}


def plan_spawn_from_np_random(rs):
    """np.random draws of plan_waypoint_env.py:205-206 (distance, heading per waypoint)
    -> [dis0..4, hdg0..4]."""
    d, h = [], []
    for _ in range(P_NUM_WAYPOINTS):
        d.append(float(rs.randint(P_WAYPOINT_DISTANCE_MIN, P_WAYPOINT_DISTANCE_MAX)))
        h.append(float(rs.randint(0, 359)))
    return np.array(d + h, np.float64)
