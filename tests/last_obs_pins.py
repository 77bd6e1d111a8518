"""Value-level pins of the sim layer from the observations the reference's saved models hold
(tests/golden/last_obs.npz, written by tests/golden/extract_last_obs.py from the plain-JSON
``data`` member of ``scripts/common/results/models_backup/*/model.zip``; no unpickling).

An off-policy model (SAC / DDPG) holds two consecutive observations of the reference's own
simulator, ``last_original_obs`` (before its last training step) and ``last_obs`` (after
it); an on-policy model (PPO) holds ``last_obs`` only.  Each value is printed with 8
decimals (``PRINT_ABS``), so a reconstructed quantity carries that precision times the
env's normalisation scale.  What they pin:

* MergeEnv-v0 (merge_env.py:191, 221-234): the ownship's TAS at 10,000 m (239.5705319 m/s =
  Mach 0.80, the perf model's Mmo) and, through the relative velocities of the two SAC
  observations, every intruder's speed (the same Mach cap: the logged stream was created at
  a CAS above the cap's 147 m/s, not merge_env.py:30's 100);
* DescentEnv-v0 / VerticalCREnv-v0 (descent_env.py:97-115, vertical_cr_env.py:113-181): one
  30-substep step of altitude, vertical speed and runway distance -- the vertical-speed
  slew, the altitude integration, CAS 150 -> TAS at altitude and the position update;
  Vertical's ``y_difference_speed`` adds the ownship's ground-speed change;
* HorizontalCREnv-v0 (horizontal_cr_env.py:176-184): every aircraft's ground speed, which
  is the phase-GD speed cap (aircraft created at alt 0);
* SectorCREnv-v0 (sector_cr_env.py:269-303): the intruders' speed and the ownship's speed
  change and displacement over one 5-substep step.

Test infrastructure only (the oracle is imported by the callers, never by the product).
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PRINT_ABS = 5e-9            # NumPy's default print precision: 8 decimals
BEFORE, AFTER = "last_original_obs", "last_obs"

# normalisations of the reference envs
MERGE_V = 150.0                                   # merge_env.py:229-230 (vx_r, vy_r /150)
ALT_MEAN, ALT_STD, VZ_STD = 1500.0, 3000.0, 5.0   # descent_env.py:12-15, vertical_cr_env.py:24-27
RWY_MEAN, RWY_STD = 100.0, 200.0                  # descent_env.py:16-17
AC_SPD_VH = 150.0                                 # vertical_cr_env.py:40, horizontal_cr_env.py:26
SECTOR_X, SECTOR_VX, SECTOR_VY = 13000.0, 32.0, 66.0   # sector_cr_env.py:300-303


def load():
    return dict(np.load(os.path.join(HERE, "golden", "last_obs.npz")))


def obs(L, env, alg, which=AFTER):
    pre = f"{env}/{alg}/{which}/"
    return {k[len(pre):]: v for k, v in L.items() if k.startswith(pre)}


# ---- MergeEnv-v0 ----------------------------------------------------------------------
def merge_intruder_speeds(L, alg="SAC"):
    """The ownship's headings (h0, h1) from the two SAC observations, given its speed (obs
    ``airspeed``, raw TAS): an intruder that is the same aircraft in both top-5 lists and flies
    a straight LNAV leg at constant velocity changes its relative velocity by exactly the
    ownship's velocity change, a chord of the circle |v| = airspeed.  The chord fixes
    the turn; its two mirror solutions are told apart by the scenario: every Merge aircraft
    flies south (spawned on +-15 deg radials north of FIX, FIX 200 km north of RWY;
    merge_env.py:42-44, 118-120, 148-158).  Every listed intruder's velocity at both steps is
    then its relative velocity plus the ownship's.  Returns (intruder speeds [2, 5], ownship
    headings [2] deg, the steady intruders, max spread of their heading solutions deg)."""
    o = [obs(L, "MergeEnv-v0", alg, w) for w in (BEFORE, AFTER)]
    v0 = [float(x["airspeed"][0]) for x in o]
    vr = [np.stack([x["vx_r"], x["vy_r"]], 1) * MERGE_V for x in o]
    chord = vr[0] - vr[1]                   # v_own(t+1) - v_own(t) for a steady intruder
    steady = np.flatnonzero(np.hypot(*(chord - np.median(chord, 0)).T) < 1e-3)
    sols = []
    for i in steady:
        c = chord[i]
        rot = 2.0 * np.arcsin(np.hypot(*c) / (v0[0] + v0[1]))
        d = np.arctan2(c[1], c[0])
        for hm in (d + np.pi / 2, d - np.pi / 2):
            for s in (1.0, -1.0):
                h = np.array([hm - s * rot / 2, hm + s * rot / 2])
                e = (v0[1] * np.array([np.cos(h[1]), np.sin(h[1])]) -
                     v0[0] * np.array([np.cos(h[0]), np.sin(h[0])]) - c)
                if np.abs(e).max() < 1e-6 and np.cos(h[1]) < 0.0:      # southbound
                    sols.append(h)
    sols = np.array(sols)
    h = sols.mean(0)
    speeds = np.stack([np.hypot(*(vr[t] + v0[t] * np.array([np.cos(h[t]), np.sin(h[t])])).T)
                       for t in range(2)])
    return speeds, np.degrees(h) % 360.0, steady, float(np.degrees(np.ptp(sols, 0)).max())


# ---- DescentEnv-v0 / VerticalCREnv-v0 ---------------------------------------------------
def vertical_ownship(L, env, alg, which):
    """(alt m, vs m/s, runway distance km, target alt m) from a Descent / Vertical obs."""
    o = obs(L, env, alg, which)
    return dict(alt=ALT_MEAN + ALT_STD * float(o["altitude"][0]),
                vs=VZ_STD * float(o["vz"][0]),
                rd=RWY_MEAN + RWY_STD * float(o["runway_distance"][0]),
                tgt=ALT_MEAN + ALT_STD * float(o["target_altitude"][0]))


def implied_action(L, env, alg):
    """The action whose selvs (a * 12.5 m/s, descent_env.py:146-160) the ownship holds at the
    end of the step (the slew reaches it within the step in both saved transitions)."""
    return vertical_ownship(L, env, alg, AFTER)["vs"] / 12.5


def ownship_start(bsx, t0, rwy=(52.0, 4.0)):
    """A single-aircraft state reproducing observation t0: on the meridian north of the
    runway at the observed distance, heading 0 (cre's default heading; the distance from the
    runway grows by the TAS whichever constant heading), CAS 150 held (descent_env.py:173)
    with the TAS of the previous substep's altitude, the observed vertical speed."""
    lat = rwy[0] + np.degrees((200.0 - t0["rd"]) * 1000.0 / bsx.Rearth)
    alt_prev = t0["alt"] - t0["vs"]
    return dict(lat=lat, lon=rwy[1], alt=t0["alt"], hdg=0.0, tas=float(bsx.vcas2tas(150.0, alt_prev)),
                cas=150.0, vs=t0["vs"], selspd=150.0)


def oracle_step(bsx, start, action, n=30, dt=1.0, rwy=(52.0, 4.0)):
    """n oracle substeps of the start state under the vertical action (descent_env.py:146-160);
    returns (alt, vs, rd km, tas)."""
    st = bsx.TrafState((1,))
    bsx.cre_state(st, 0, start["lat"], start["lon"], start["hdg"], start["alt"], start["cas"])
    st.tas[0], st.vs[0], st.selspd[0] = start["tas"], start["vs"], start["selspd"]
    st.selalt[0] = 1e6 if action >= 0 else 0.0
    st.selvs[0] = action * 12.5
    for _ in range(n):
        bsx.traffic_update(st, dt, [], [], [])
    rd = 200.0 - float(bsx.kwikdist(rwy[0], rwy[1], st.lat[0], st.lon[0])) * 1.852
    return dict(alt=float(st.alt[0]), vs=float(st.vs[0]), rd=rd, tas=float(st.tas[0]))


def vertical_ydif_change(L, alg="SAC"):
    """VerticalCREnv y_difference_speed = gs_own - sin(dhdg) gs_int (vertical_cr_env.py:149):
    its change over the step, per intruder (level intruders on constant headings), is the
    ownship's ground-speed change [m/s]."""
    o = [obs(L, "VerticalCREnv-v0", alg, w) for w in (BEFORE, AFTER)]
    return (o[1]["y_difference_speed"] - o[0]["y_difference_speed"]) * AC_SPD_VH


# ---- HorizontalCREnv-v0 -----------------------------------------------------------------
def horizontal_common_speed(L, alg, which):
    """x_dif = -cos(dhdg) gs_i, y_dif = gs_0 - sin(dhdg) gs_i (horizontal_cr_env.py:180-181):
    with one speed g for every aircraft, g = (x_dif^2 + y_dif^2) / (2 y_dif) per intruder."""
    o = obs(L, "HorizontalCREnv-v0", alg, which)
    x = o["x_difference_speed"] * AC_SPD_VH
    y = o["y_difference_speed"] * AC_SPD_VH
    return (x * x + y * y) / (2.0 * y)


# ---- SectorCREnv-v0 ---------------------------------------------------------------------
def _chord_headings(v0, v1, c):
    """Both pairs (h0, h1) with v1 u(h1) - v0 u(h0) = c (u = unit vector north/east)."""
    out = []
    # |c|^2 = v0^2 + v1^2 - 2 v0 v1 cos(h1 - h0); the chord's direction fixes the rest
    cosd = np.clip((v0 * v0 + v1 * v1 - c @ c) / (2.0 * v0 * v1), -1.0, 1.0)
    for dh in (np.arccos(cosd), -np.arccos(cosd)):
        # c = R(h0) [v1 u(dh) - v0 u(0)]  ->  h0 = angle(c) - angle(v1 u(dh) - v0 u(0))
        w = np.array([v1 * np.cos(dh) - v0, v1 * np.sin(dh)])
        h0 = np.arctan2(c[1], c[0]) - np.arctan2(w[1], w[0])
        out.append(np.array([h0, h0 + dh]))
    return out


def sector_transition(L, alg="SAC"):
    """The SAC transition of SectorCREnv: ownship speeds (obs airspeed = (tas - 150) / 6),
    its velocity change (minus the change of every intruder's relative velocity: the four
    agree to 1e-6, so they fly constant velocities), its headings, each intruder's speed, and
    the ownship's north displacement over the step estimated from each intruder (relative
    north displacement through latlong_to_nm's 60 NM per degree, functions.py, against the
    simulator's Rearth).  Of the two mirror heading solutions the one is taken on which the
    intruders -- one type, one altitude, one creation speed, no speed commands
    (sector_cr_env.py:217) -- share one speed; the other spreads them over 69-110 m/s."""
    o = [obs(L, "SectorCREnv-v0", alg, w) for w in (BEFORE, AFTER)]
    v = [float(x["airspeed"][0]) * 6.0 + 150.0 for x in o]
    vr = [np.stack([x["vx_r"] * SECTOR_VX, x["vy_r"] * SECTOR_VY], 1) for x in o]
    dv_each = -(vr[1] - vr[0])
    best = None
    for h in _chord_headings(v[0], v[1], dv_each.mean(0)):
        own1 = v[1] * np.array([np.cos(h[1]), np.sin(h[1])])
        vint = vr[1] + own1
        spd = np.hypot(vint[:, 0], vint[:, 1])
        if best is None or np.ptp(spd) < np.ptp(best[1]):
            best = (h, spd, vint)
    h, spd, vint = best
    scale = 60.0 * 1852.0 / (np.pi / 180.0 * 6371000.0)
    dx_real = (o[1]["x_r"] - o[0]["x_r"]) * SECTOR_X / scale
    own_north = 5.0 * vint[:, 0] - dx_real
    return dict(speeds=v, dv_each=dv_each, headings=np.degrees(h) % 360.0,
                intruder_speeds=spd, own_north=own_north)
