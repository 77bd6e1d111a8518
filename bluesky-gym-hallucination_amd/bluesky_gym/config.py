"""Frozen per-env-kind configuration.  Defaults are the reference's module constants.

Merge:    bluesky_gym/envs/merge_env.py:13-46  (NUM_AC=20, NUM_AC_STATE=5,
          ACTION_FREQUENCY=10, 'DT 5' at :86, TimeLimit 50 at bluesky_gym/__init__.py:45)
Vertical: bluesky_gym/envs/vertical_cr_env.py:12-45 (NUM_INTRUDERS=5 -- redefined at :45,
          ACTION_FREQUENCY=30, 'DT 1' at :95, TimeLimit 300 at __init__.py:27)
Descent:  bluesky_gym/envs/descent_env.py:10-30 (ACTION_FREQUENCY=30, 'DT 1' at :72,
          TimeLimit 300 at __init__.py:9)
HorizontalCR: bluesky_gym/envs/horizontal_cr_env.py:11-30 (NUM_INTRUDERS=5,
          ACTION_FREQUENCY=10, 'DT 5' at :71, TimeLimit 300 at __init__.py:19-22)
StaticObstacle: bluesky_gym/envs/static_obstacle_env.py:12-41 (ACTION_FREQUENCY=10,
          'DT 1' at :85, TimeLimit 100 at __init__.py:36-40)
SectorCR: bluesky_gym/envs/sector_cr_env.py:11-38 (ACTION_FREQUENCY=5, NUM_AC_STATE=4,
          'DT 1' at :78, TimeLimit 200 at __init__.py:30-34); the aircraft count is drawn
          per episode, num_ac is the capacity of an env (default 32)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _native as nat

# merge_env.py:41-46 -- FIX is computed exactly as the reference does at import time
RWY_LAT = 52.36239301495972
RWY_LON = 4.713195734579777


def get_point_at_distance(lat1, lon1, d, bearing, R=6371):
    """functions.py:24-42 (great-circle destination, d in km)."""
    lat1 = np.radians(lat1)
    lon1 = np.radians(lon1)
    a = np.radians(bearing)
    lat2 = np.arcsin(np.sin(lat1) * np.cos(d / R) + np.cos(lat1) * np.sin(d / R) * np.cos(a))
    lon2 = lon1 + np.arctan2(np.sin(a) * np.sin(d / R) * np.cos(lat1),
                             np.cos(d / R) - np.sin(lat1) * np.sin(lat2))
    return float(np.degrees(lat2)), float(np.degrees(lon2))


def _rwgs84(latd):
    lat = np.radians(latd)
    a, b = 6378137.0, 6356752.314245
    coslat, sinlat = np.cos(lat), np.sin(lat)
    an, bn, ad, bd = a * a * coslat, b * b * sinlat, a * coslat, b * sinlat
    return np.sqrt((an * an + bn * bn) / (ad * ad + bd * bd))


def wgs84_bearing(latd1, lond1, latd2, lond2):
    """bluesky.tools.geo.qdrdist bearing (deg) -- used once for the route's leg bearing."""
    lat1, lon1, lat2, lon2 = (np.radians(v) for v in (latd1, lond1, latd2, lond2))
    coslat1, coslat2 = np.cos(lat1), np.cos(lat2)
    return float(np.degrees(np.arctan2(np.sin(lon2 - lon1) * coslat2,
                                       coslat1 * np.sin(lat2) -
                                       np.sin(lat1) * coslat2 * np.cos(lon2 - lon1))))


FIX_LAT, FIX_LON = get_point_at_distance(RWY_LAT, RWY_LON, 200, 0)


@dataclass(frozen=True)
class EnvKindConfig:
    kind: int
    num_ac: int
    num_ac_state: int
    action_frequency: int
    simdt: float
    max_episode_steps: int
    kind_option: int = 0
    # MergeEnv-v0: its module constants (_native.MERGE_PARAMS order), () = the reference's
    params: tuple = ()

    def to_c(self, num_envs, autoreset, compute_cd, seed, device, env_offset=0) -> nat.BsgConfig:
        c = nat.BsgConfig()
        c.abi_version = nat.ABI_VERSION
        c.env_kind = self.kind
        c.num_envs = int(num_envs)
        c.num_ac = int(self.num_ac)
        c.num_ac_state = int(self.num_ac_state)
        c.action_frequency = int(self.action_frequency)
        c.simdt = float(self.simdt)
        c.max_episode_steps = int(self.max_episode_steps)
        c.autoreset_mode = int(autoreset)
        c.compute_cd = int(bool(compute_cd))
        c.device = int(device)
        c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        c.env_offset = int(env_offset)
        c.kind_option = int(self.kind_option)
        if self.kind == nat.ENV_MERGE:
            # ADDWPT FIX ; DEST RWY (merge_env.py:155-156)
            c.route_len = 2
            c.route_lat[0], c.route_lon[0] = FIX_LAT, FIX_LON
            c.route_lat[1], c.route_lon[1] = RWY_LAT, RWY_LON
            c.route_next_qdr[0] = wgs84_bearing(FIX_LAT, FIX_LON, RWY_LAT, RWY_LON)
            c.route_next_qdr[1] = -999.0
            c.wpt_lat[0], c.wpt_lon[0] = FIX_LAT, FIX_LON
            c.wpt_lat[1], c.wpt_lon[1] = RWY_LAT, RWY_LON
        return c


def merge_config(num_ac=20, num_ac_state=5, action_frequency=10, simdt=5.0,
                 max_episode_steps=50, ac_spd=None, params=None):
    """ac_spd: creation CAS [m/s] of every aircraft (merge_env.py:30 AC_SPD); None = 100.
    params: {name: value} for any of merge_env.py:13-28's D_HEADING, D_SPEED,
    INTRUSION_DISTANCE, DISTANCE_MARGIN, REACH_REWARD, DRIFT_PENALTY, INTRUSION_PENALTY,
    SPAWN_DISTANCE_MIN/MAX, INTRUDER_DISTANCE_MIN/MAX (the others keep the reference's
    values); handed to the kernel by bsg_set_params."""
    opt = 0 if ac_spd is None or int(ac_spd) == 100 else int(ac_spd)
    if ac_spd is not None and float(ac_spd) != int(ac_spd):
        raise ValueError("ac_spd must be a whole number of m/s")
    vals = ()
    if params:
        names = [n for n, _ in nat.MERGE_PARAMS]
        bad = set(params) - set(names)
        if bad:
            raise ValueError(f"merge_config: unknown params {sorted(bad)}; known {names}")
        full = [float(params.get(n, v)) for n, v in nat.MERGE_PARAMS]
        if full != [v for _, v in nat.MERGE_PARAMS]:
            vals = tuple(full)
    return EnvKindConfig(nat.ENV_MERGE, num_ac, num_ac_state, action_frequency, simdt,
                         max_episode_steps, opt, vals)


def vertical_config(num_intruders=5, action_frequency=30, simdt=1.0, max_episode_steps=300):
    return EnvKindConfig(nat.ENV_VERTICAL_CR, num_intruders + 1, 0, action_frequency, simdt,
                         max_episode_steps)


def horizontal_config(num_intruders=5, action_frequency=10, simdt=5.0, max_episode_steps=300):
    return EnvKindConfig(nat.ENV_HORIZONTAL_CR, num_intruders + 1, 0, action_frequency, simdt,
                         max_episode_steps)


def static_config(action_frequency=10, simdt=1.0, max_episode_steps=100):
    return EnvKindConfig(nat.ENV_STATIC_OBSTACLE, 1, 0, action_frequency, simdt, max_episode_steps)


def sector_config(num_ac=32, action_frequency=5, simdt=1.0, max_episode_steps=200,
                  density_mode="normal"):
    if density_mode not in ("normal", "uniform"):
        raise ValueError("density_mode must be 'normal' or 'uniform' (sector_cr_env.py:95-100)")
    return EnvKindConfig(nat.ENV_SECTOR_CR, num_ac, 4, action_frequency, simdt, max_episode_steps,
                         0 if density_mode == "normal" else 1)


def descent_config(action_frequency=30, simdt=1.0, max_episode_steps=300):
    return EnvKindConfig(nat.ENV_DESCENT, 1, 0, action_frequency, simdt, max_episode_steps)


def plan_waypoint_config(action_frequency=10, simdt=1.0, max_episode_steps=300):
    """plan_waypoint_env.py:21 ACTION_FREQUENCY, :72 'DT 1', bluesky_gym/__init__.py:15."""
    return EnvKindConfig(nat.ENV_PLAN_WAYPOINT, 1, 0, action_frequency, simdt, max_episode_steps)
