"""Host-side spawn draws that consume Python ``random`` / legacy ``np.random`` exactly as
the reference envs do, so ``random.seed(s); env.reset()`` reproduces the reference's
episode start (parity mode).  The device (Philox) draw is the throughput default of the
vector envs.

merge_env.py:115-116 + _gen_aircraft :150-151   (random.uniform, 2 + 2*(N-1) draws)
vertical_cr_env.py:267-268 + :187-195          (np.random.randint, 2 + 4*(N-1) draws)
descent_env.py:170-171                         (np.random.randint, 2 draws)
horizontal_cr_env.py:130-132 + :140            (np.random.randint, 3*(N-1) + 1 draws)
"""
from __future__ import annotations

import random as _random

import numpy as np

D_HEADING = 15
SPAWN_DISTANCE_MIN, SPAWN_DISTANCE_MAX = 50, 200
INTRUDER_DISTANCE_MIN, INTRUDER_DISTANCE_MAX = 20, 500
ALT_MIN, ALT_MAX = 2000, 4000
TARGET_ALT_DIF = 500
DEFAULT_RWY_DIS = 200
ACTION_2_MS = 12.5
V_AC_SPD = 150
INTRUSION_DISTANCE_NM = 5
H_WAYPOINT_DISTANCE_MIN, H_WAYPOINT_DISTANCE_MAX = 100, 150

# bluesky.tools.aero constants (for the reference's randint bound, vertical_cr_env.py:190)
_P0, _RHO0, _R = 101325.0, 1.225, 287.05287


def _vcas2tas(cas, h):
    """bluesky.tools.aero.vcas2tas (ISA) on the host: the ownship ground speed that the
    reference reads back after cre() to bound tlosh."""
    T = np.maximum(288.15 - 0.0065 * h, 216.65)
    rho = 1.225 * (T / 288.15) ** 4.256848030018761 * np.exp(-np.maximum(0.0, h - 11000.0) / 6341.552161)
    p = rho * _R * T
    qdyn = _P0 * ((1.0 + _RHO0 * cas * cas / (7.0 * _P0)) ** 3.5 - 1.0)
    tas = np.sqrt(7.0 * p / rho * ((1.0 + qdyn / p) ** (2.0 / 7.0) - 1.0))
    return np.where(cas < 0, -1 * tas, tas)


def merge_spawn(num_ac, rng=None, d_heading=None, spawn_range=None, intruder_range=None):
    """d_heading / spawn_range / intruder_range: merge_env.py's D_HEADING,
    SPAWN_DISTANCE_MIN/MAX, INTRUDER_DISTANCE_MIN/MAX (None: the reference's values)."""
    rng = _random if rng is None else rng
    dh = D_HEADING if d_heading is None else d_heading
    s0, s1 = (SPAWN_DISTANCE_MIN, SPAWN_DISTANCE_MAX) if spawn_range is None else spawn_range
    i0, i1 = (INTRUDER_DISTANCE_MIN, INTRUDER_DISTANCE_MAX) if intruder_range is None else intruder_range
    out = [rng.uniform(-dh, dh), rng.uniform(s0, s1)]
    for _ in range(num_ac - 1):
        out.append(rng.uniform(-dh, dh))
        out.append(rng.uniform(i0, i1))
    return np.array(out, np.float64)


def vertical_spawn(num_intruders, rs=None):
    rs = np.random if rs is None else rs
    alt_init = rs.randint(ALT_MIN, ALT_MAX)
    target_alt = alt_init + rs.randint(-TARGET_ALT_DIF, TARGET_ALT_DIF)
    altitude = float(alt_init)
    spd = float(_vcas2tas(np.float64(V_AC_SPD), np.float64(alt_init)))
    out = [float(alt_init), float(target_alt)]
    for _ in range(num_intruders):
        dpsi = rs.randint(45, 315)
        cpa = rs.randint(0, INTRUSION_DISTANCE_NM)
        tlosh = rs.randint(100, int((DEFAULT_RWY_DIS * 0.9) * 1000 / spd))
        average_tod = (DEFAULT_RWY_DIS * 1000 / spd) - 2 * target_alt / ACTION_2_MS
        if tlosh > average_tod:
            dH = rs.randint(int(-altitude + 500), int((target_alt - altitude) + 100))
        else:
            dH = rs.randint(int((target_alt - altitude) - 500), int((target_alt - altitude) + 500))
        out += [float(dpsi), float(cpa), float(tlosh), float(dH)]
    return np.array(out, np.float64)


def horizontal_spawn(num_intruders, rs=None):
    rs = np.random if rs is None else rs
    out = []
    for _ in range(num_intruders):
        dpsi = rs.randint(45, 315)
        cpa = rs.randint(0, INTRUSION_DISTANCE_NM)
        tlosh = rs.randint(100, 1000)
        out += [float(dpsi), float(cpa), float(tlosh)]
    out.append(float(rs.randint(H_WAYPOINT_DISTANCE_MIN, H_WAYPOINT_DISTANCE_MAX)))
    return np.array(out, np.float64)


def plan_spawn(rs=None):
    """np.random draws of plan_waypoint_env.py:205-206, per waypoint (distance km, bearing
    deg) -> [dis0..4, hdg0..4] (the PlanWaypoint spawn row, bsg.h bsg_spawn_width)."""
    rs = np.random if rs is None else rs
    d, h = [], []
    for _ in range(5):
        d.append(float(rs.randint(0, 75)))
        h.append(float(rs.randint(0, 359)))
    return np.array(d + h, np.float64)


def descent_spawn(rs=None):
    rs = np.random if rs is None else rs
    alt_init = rs.randint(ALT_MIN, ALT_MAX)
    target_alt = alt_init + rs.randint(-TARGET_ALT_DIF, TARGET_ALT_DIF)
    return np.array([float(alt_init), float(target_alt)], np.float64)
