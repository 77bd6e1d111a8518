"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- StaticObstacleEnv-v0 and SectorCREnv-v0 in the
batched form of oracle/batched.py (envs as rows, aircraft as columns).

static_obstacle_env.py (:96-345) and sector_cr_env.py (:84-339) restated on top of the
BlueSky subset (oracle/bluesky_subset.py) and the polygon helpers (oracle/areas.py);
pinned against the reference env code by tests/golden/{static,sector}_*.npz.
"""
from __future__ import annotations

import numpy as np

from . import areas
from . import bluesky_subset as bsx
from .batched import (AUTORESET_NEXT_STEP, NM2KM, _Base, _rows_to_u64, flatten_obs)

STATIC_OBS_KEYS = ("cos_difference_restricted_area_pos", "destination_waypoint_cos_drift",
                   "destination_waypoint_distance", "destination_waypoint_sin_drift",
                   "restricted_area_distance", "restricted_area_radius",
                   "sin_difference_restricted_area_pos")
SECTOR_OBS_KEYS = ("airspeed", "cos(drift)", "cos(track)", "distances", "sin(drift)",
                   "sin(track)", "vx_r", "vy_r", "x_r", "y_r")

# static_obstacle_env.py:12-41
S_DISTANCE_MARGIN = 5
S_REACH_REWARD = 1
S_DRIFT_PENALTY = -0.01
S_RA_INTRUSION_PENALTY = -5
S_WAYPOINT_DISTANCE_MAX = 170
S_D_HEADING = 45
S_D_SPEED = 20 / 3
S_AC_SPD = 150
S_ALTITUDE = 350
MPS2KT = 1.94384
NOBST = areas.STATIC_NUM_OBSTACLES

# sector_cr_env.py:11-38
C_AC_SPD = 150
C_ALTITUDE = 350
C_INTRUSION_DISTANCE = 5
C_NUM_AC_STATE = 4
C_DRIFT_PENALTY = -0.1
C_INTRUSION_PENALTY = -1
C_D_HEADING = 22.5
C_D_VELOCITY = 20 / 3


def static_obs_sizes():
    return {"cos_difference_restricted_area_pos": NOBST, "destination_waypoint_cos_drift": 1,
            "destination_waypoint_distance": 1, "destination_waypoint_sin_drift": 1,
            "restricted_area_distance": NOBST, "restricted_area_radius": NOBST,
            "sin_difference_restricted_area_pos": NOBST}


def sector_obs_sizes(k=C_NUM_AC_STATE):
    return {"airspeed": 1, "cos(drift)": 1, "cos(track)": k, "distances": k, "sin(drift)": 1,
            "sin(track)": k, "vx_r": k, "vy_r": k, "x_r": k, "y_r": k}


def _hdg_spd_action(o, actions, d_heading, d_speed):
    """HDG / SPD stack commands of the ownship (static_obstacle_env.py:339-346,
    sector_cr_env.py:313-320)."""
    st = o.st
    heading_new = bsx.bound_angle_positive_negative_180(st.hdg[:, 0] + actions[:, 0] * d_heading)
    speed_new = (st.cas[:, 0] + actions[:, 1] * d_speed) * MPS2KT
    st.ap_trk[:, 0] = bsx.selhdg_track(st, (slice(None), 0), heading_new, o.wind)
    st.swlnav[:, 0] = False
    st.selspd[:, 0] = np.where(speed_new >= 1.0, speed_new * bsx.kts, speed_new)


class StaticOracle(_Base):
    """StaticObstacleEnv-v0: one aircraft, NUM_OBSTACLES restricted-area polygons."""
    kind = "static"

    def __init__(self, num_envs, action_frequency=10, simdt=1.0, max_episode_steps=100,
                 autoreset=AUTORESET_NEXT_STEP, seed=0):
        super().__init__(num_envs, 1, action_frequency, simdt, max_episode_steps, autoreset, seed)
        E = self.E
        self.clat = np.zeros((E, NOBST))
        self.clon = np.zeros((E, NOBST))
        self.R = np.zeros((E, NOBST))
        self.polys = [[(np.zeros(3), np.zeros(3))] * NOBST for _ in range(E)]
        self.wlat = np.zeros(E)
        self.wlon = np.zeros(E)
        self.wpt_reach = np.zeros(E, np.int32)
        self.waypoint_reached = np.zeros(E, np.int32)
        self.crashed = np.zeros(E, np.int32)
        self.drift_sum = np.zeros(E)
        self.drift_cnt = np.zeros(E, np.int64)
        self.last_wdist = np.zeros(E)        # destination_waypoint_distance of the last obs (km)
        self.last_drift = np.zeros(E)        # destination_waypoint_drift of the last obs (deg)
        self.obs_sizes = static_obs_sizes()
        self.obs_dim = sum(self.obs_sizes.values())

    def spawn_width(self):
        return NOBST * (4 + areas.STATIC_VMAX) + 2

    def device_spawn_params(self, env_ids, episodes):
        return np.stack([areas.static_device_spawn(int(e), int(ep), self.seed)
                         for e, ep in zip(env_ids, episodes)])

    def _reset_ids(self, ids, spawn):
        """static_obstacle_env.py:96-124."""
        st = self.st
        for e in ids:
            g = areas.static_polygons(spawn[e])
            self.clat[e], self.clon[e], self.R[e] = g["clat"], g["clon"], g["R"]
            self.polys[e] = g["poly"]
            self.wlat[e], self.wlon[e] = g["wpt"]
            bsx.cre_state(st, (e, 0), 52.0, 4.0, 0.0, S_ALTITUDE, S_AC_SPD)
            qdr, _ = bsx.kwikqdrdist(st.lat[e, 0], st.lon[e, 0], self.wlat[e], self.wlon[e])
            st.hdg[e, 0] = qdr
            st.ap_trk[e, 0] = qdr
        self.wpt_reach[ids] = 0
        self.waypoint_reached[ids] = 0
        self.crashed[ids] = 0
        self.drift_sum[ids] = 0.0
        self.drift_cnt[ids] = 0
        _, wd, dr = self._own_terms()
        self.last_wdist[ids] = wd[ids]
        self.last_drift[ids] = dr[ids]

    def _apply_action(self, actions):
        _hdg_spd_action(self, actions, S_D_HEADING, S_D_SPEED)

    def _inside_count(self):
        st = self.st
        n = np.zeros(self.E, np.int32)
        for e in range(self.E):
            for o in range(NOBST):
                pl = self.polys[e][o]
                n[e] += int(areas.points_in_poly(st.lat[e, 0], st.lon[e, 0], pl[0], pl[1]))
        return n

    def step(self, actions, spawn=None):
        self._live = ~self.needs_reset if self.autoreset == AUTORESET_NEXT_STEP \
            else np.ones(self.E, bool)
        return super().step(actions, spawn)

    def _substeps(self):
        """static_obstacle_env.py:132-150: _get_reward after every substep with the
        waypoint distance / drift of the LAST observation; stop at the first done."""
        E = self.E
        going = np.ones(E, bool)
        wr = self.wpt_reach.copy()
        wreached = self.waypoint_reached.copy()
        crashed = self.crashed.copy()
        dsum = self.drift_sum.copy()
        dcnt = self.drift_cnt.copy()
        reward = np.zeros(E)
        done = np.zeros(E, bool)
        for _ in range(self.S):
            pre = self.st.copy()
            bsx.traffic_update(self.st, self.dt, self.route_lat, self.route_lon,
                               self.route_next_qdr, self.wind)
            for f in bsx.FIELDS_F64:
                getattr(self.st, f)[~going] = getattr(pre, f)[~going]
            reach = going & (self.last_wdist < S_DISTANCE_MARGIN) & (wr != 1)
            wr = np.where(reach, 1, wr)
            wreached = np.where(reach, 1, wreached)
            dd = np.abs(np.deg2rad(self.last_drift))
            dsum = np.where(going, dsum + dd, dsum)
            dcnt = dcnt + going
            nin = self._inside_count()
            crashed = np.where(going & (nin > 0), 1, crashed)
            r = (np.where(reach, S_REACH_REWARD, 0) + dd * S_DRIFT_PENALTY) + \
                nin * S_RA_INTRUSION_PENALTY
            reward = np.where(going, r, reward)
            d = going & ((wr == 1) | (nin > 0))
            done |= d
            going &= ~d
        self._sub = dict(wr=wr, wreached=wreached, crashed=crashed, dsum=dsum, dcnt=dcnt,
                         reward=reward, done=done)

    def _own_terms(self):
        st = self.st
        hdg = st.hdg[:, 0]
        wqdr, wdis = bsx.kwikqdrdist(st.lat[:, 0], st.lon[:, 0], self.wlat, self.wlon)
        drift = bsx.bound_angle_positive_negative_180(hdg - wqdr)
        cqdr, cdis = bsx.kwikqdrdist(st.lat[:, :1], st.lon[:, :1], self.clat, self.clon)
        bearing = bsx.bound_angle_positive_negative_180(hdg[:, None] - cqdr)
        obs = {
            "destination_waypoint_distance": ((wdis * NM2KM) / S_WAYPOINT_DISTANCE_MAX)[:, None],
            "destination_waypoint_cos_drift": np.cos(np.deg2rad(drift))[:, None],
            "destination_waypoint_sin_drift": np.sin(np.deg2rad(drift))[:, None],
            "restricted_area_radius": self.R / 50,
            "restricted_area_distance": (cdis * NM2KM) / S_WAYPOINT_DISTANCE_MAX,
            "cos_difference_restricted_area_pos": np.cos(np.deg2rad(bearing)),
            "sin_difference_restricted_area_pos": np.sin(np.deg2rad(bearing)),
        }
        return obs, wdis * NM2KM, drift

    def observe(self):
        obs, _, _ = self._own_terms()
        return {"obs": self._flat(obs, STATIC_OBS_KEYS), "obs_dict": obs}

    def _observe_and_reward(self):
        obs, wd, dr = self._own_terms()
        self._obs_terms = (wd, dr)
        return dict(obs=self._flat(obs, STATIC_OBS_KEYS), obs_dict=obs, reward=self._sub["reward"],
                    terminated=self._sub["done"], intr_mask=np.zeros(self.E, np.uint64),
                    nintr=np.zeros(self.E, np.int32))

    def _commit(self, res, live):
        s = self._sub
        for name, key in (("wpt_reach", "wr"), ("waypoint_reached", "wreached"),
                          ("crashed", "crashed"), ("drift_sum", "dsum"), ("drift_cnt", "dcnt")):
            setattr(self, name, np.where(live, s[key], getattr(self, name)))
        wd, dr = self._obs_terms
        self.last_wdist = np.where(live, wd, self.last_wdist)
        self.last_drift = np.where(live, dr, self.last_drift)
        self.total_reward = np.where(live, self.total_reward + res["reward"], self.total_reward)

    def info(self):
        with np.errstate(invalid="ignore", divide="ignore"):
            avg = self.drift_sum / self.drift_cnt
        return {"total_reward": self.total_reward.copy(),
                "waypoint_reached": self.waypoint_reached.copy(),
                "crashed": self.crashed.copy(),
                "average_drift": np.where(self.drift_cnt > 0, avg, np.nan)}


class SectorOracle(_Base):
    """SectorCREnv-v0: a random sector polygon with a random number of aircraft (<= N)."""
    kind = "sector"

    def __init__(self, num_envs, num_ac=32, action_frequency=5, simdt=1.0, max_episode_steps=200,
                 autoreset=AUTORESET_NEXT_STEP, seed=0, compute_cd=True, density_mode="normal"):
        super().__init__(num_envs, num_ac, action_frequency, simdt, max_episode_steps, autoreset,
                         seed)
        E = self.E
        self.K = C_NUM_AC_STATE
        self.compute_cd = compute_cd
        self.density_mode = density_mode
        self.nac = np.full(E, self.N, np.int32)
        self.plat = [np.zeros(3)] * E
        self.plon = [np.zeros(3)] * E
        self.wlat = np.zeros(E)
        self.wlon = np.zeros(E)
        self.drift_sum = np.zeros(E)
        self.drift_cnt = np.zeros(E, np.int32)
        self.obs_sizes = sector_obs_sizes()
        self.obs_dim = sum(self.obs_sizes.values())

    def spawn_width(self):
        return 4 + 2 * areas.SECTOR_VMAX + 3 * self.N

    def device_spawn_params(self, env_ids, episodes):
        return np.stack([areas.sector_device_spawn(int(e), int(ep), self.seed, self.N,
                                                   self.density_mode)
                         for e, ep in zip(env_ids, episodes)])

    def _reset_ids(self, ids, spawn):
        """sector_cr_env.py:84-109, _generate_ac :184-208."""
        st = self.st
        V = areas.SECTOR_VMAX
        base = 4 + 2 * V
        for e in ids:
            row = spawn[e]
            nac, nv = int(row[0]), int(row[1])
            self.nac[e] = nac
            self.plat[e] = row[2:2 + nv].copy()
            self.plon[e] = row[2 + V:2 + V + nv].copy()
            self.wlat[e], self.wlon[e] = row[2 + 2 * V], row[3 + 2 * V]
            for j in range(self.N):
                if j < nac:
                    lat, lon, hdg = row[base + 3 * j: base + 3 * j + 3]
                    bsx.cre_state(st, (e, j), lat, lon, hdg, C_ALTITUDE, C_AC_SPD)
                else:
                    bsx.cre_state(st, (e, j), 0.0, 0.0, 0.0, 0.0, 0.0)
        self.drift_sum[ids] = 0.0
        self.drift_cnt[ids] = 0

    def active(self):
        return np.arange(self.N)[None, :] < self.nac[:, None]

    def _apply_action(self, actions):
        _hdg_spd_action(self, actions, C_D_HEADING, C_D_VELOCITY)

    def _obs_core(self):
        """sector_cr_env.py:218-293."""
        st = self.st
        C = areas.SECTOR_CENTER
        act = self.active()
        hdg0, tas0 = st.hdg[:, 0], st.tas[:, 0]
        wqdr, _ = bsx.kwikqdrdist(st.lat[:, 0], st.lon[:, 0], self.wlat, self.wlon)
        drift = bsx.bound_angle_positive_negative_180(hdg0 - wqdr)
        vx = np.cos(np.deg2rad(hdg0)) * tas0
        vy = np.sin(np.deg2rad(hdg0)) * tas0
        cc = np.cos(np.radians(C[0]))
        x = (((st.lat - C[0]) * 60) * NM2KM) * 1000
        y = ((((st.lon - C[1]) * 60) * cc) * NM2KM) * 1000
        dx = x[:, 1:] - x[:, :1]
        dy = y[:, 1:] - y[:, :1]
        dist = np.sqrt(dx ** 2 + dy ** 2)
        dist = np.where(act[:, 1:], dist, np.inf)
        order = np.argsort(dist, axis=1, kind="stable")[:, :self.K]
        take = lambda a: np.take_along_axis(a, order, 1)
        vxi = np.cos(np.deg2rad(st.hdg[:, 1:])) * st.tas[:, 1:]
        vyi = np.sin(np.deg2rad(st.hdg[:, 1:])) * st.tas[:, 1:]
        vx_r = take(vxi) - vx[:, None]
        vy_r = take(vyi) - vy[:, None]
        track = np.arctan2(vy_r, vx_r)
        obs = {
            "cos(drift)": np.cos(np.deg2rad(drift))[:, None],
            "sin(drift)": np.sin(np.deg2rad(drift))[:, None],
            "airspeed": ((tas0 - 150) / 6)[:, None],
            "x_r": take(dx) / 13000,
            "y_r": take(dy) / 13000,
            "vx_r": vx_r / 32,
            "vy_r": vy_r / 66,
            "cos(track)": np.cos(track),
            "sin(track)": np.sin(track),
            "distances": (take(dist) - 50000.) / 15000.,
        }
        return obs, drift, order + 1

    def observe(self):
        obs, _, _ = self._obs_core()
        return {"obs": self._flat(obs, SECTOR_OBS_KEYS), "obs_dict": obs}

    def _observe_and_reward(self):
        st = self.st
        obs, drift, topk = self._obs_core()
        act = self.active()
        _, di = bsx.kwikqdrdist(st.lat[:, :1], st.lon[:, :1], st.lat[:, 1:], st.lon[:, 1:])
        intr = (di < C_INTRUSION_DISTANCE) & act[:, 1:]
        nintr = intr.sum(axis=1)
        d = np.abs(np.deg2rad(drift))
        reward = d * C_DRIFT_PENALTY + nintr * C_INTRUSION_PENALTY
        inside = np.array([bool(areas.points_in_poly(st.lat[e, 0], st.lon[e, 0], self.plat[e],
                                                     self.plon[e])) for e in range(self.E)])
        intr_mask = np.zeros(self.E, np.uint64)
        for i in range(self.N - 1):
            intr_mask |= intr[:, i].astype(np.uint64) << np.uint64(i + 1)
        res = dict(obs=self._flat(obs, SECTOR_OBS_KEYS), obs_dict=obs, reward=reward,
                   terminated=np.zeros(self.E, bool), truncated_env=~inside, intr_mask=intr_mask,
                   nintr=nintr, topk=topk, _d=d)
        if self.compute_cd:
            cd = bsx.statebased_detect(st.lat, st.lon, st.alt, st.trk, st.gs, st.vs, active=act)
            res["conf_mask"] = _rows_to_u64(cd["swconfl"])
            res["los_mask"] = _rows_to_u64(cd["swlos"])
            res["tcpamax"] = cd["tcpamax"]
            res["min_sep"] = cd["min_sep"]
            res["cd"] = cd
        return res

    def _cd_into(self, res, mask):
        st = self.st
        cd = bsx.statebased_detect(st.lat, st.lon, st.alt, st.trk, st.gs, st.vs,
                                   active=self.active())
        res["conf_mask"] = np.where(mask[:, None], _rows_to_u64(cd["swconfl"]), res["conf_mask"])
        res["los_mask"] = np.where(mask[:, None], _rows_to_u64(cd["swlos"]), res["los_mask"])
        res["tcpamax"] = np.where(mask[:, None], cd["tcpamax"], res["tcpamax"])
        res["min_sep"] = np.where(mask, cd["min_sep"], res["min_sep"])

    def _commit(self, res, live):
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
