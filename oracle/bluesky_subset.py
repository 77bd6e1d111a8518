"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- NumPy restatement of the BlueSky subset.

This module is the checker, never the product. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``bluesky_gym`` + ``libbsg.so``) never routes through here.

What it restates
----------------
The reference env layer (``/root/reference/bluesky_gym/envs/*.py``) calls into the
third-party package ``bluesky-simulator==1.0.3`` (``pyproject.toml:14``), which is NOT
vendored under ``/root/reference`` and not installed here.  This module restates the
published algorithm of the subset those call sites use (frozen in
``docs/BLUESKY_SUBSET_SPEC.md``):

* ``bluesky.tools.aero``   -- ISA atmosphere, CAS/TAS/Mach conversions
* ``bluesky.tools.geo``    -- kwikqdrdist / kwikdist / kwikdist_matrix /
                              kwikqdrdist_matrix / kwikpos / qdrdist / rwgs84
* ``bluesky.traffic``      -- Traffic.update: autopilot (HDG/SPD hold, LNAV direct-to,
                              selalt/selvs), OpenAP-style perf limits, update_airspeed,
                              update_groundspeed (no wind), update_pos
* ``bluesky.traffic.asas.statebased`` -- StateBased.detect (all-pairs CPA)
* ``bluesky.traffic.windfield``        -- WindField.addpointvne / getdata, and the wind
                              branches of ActivePilot (heading for a commanded track),
                              update_groundspeed and the HDG command (wind path, §8(f) 3)
* ``Traffic.cre`` / ``Traffic.creconfs`` (spawn)

Parity status: the SIM layer is "parity unpinned" (no upstream source or fixture is
available offline); the ENV layer built on top of it (oracle/batched.py) is pinned by
golden vectors produced by the reference's own env code (tests/golden/make_golden.py).

Every function works on arrays of any leading shape, so the same code drives the
per-env golden harness (shape [N]) and the batched oracle (shape [E, N]).
"""
from __future__ import annotations

import math

import numpy as np

# --------------------------------------------------------------------------------------
# A.1 constants (bluesky.tools.aero)
# --------------------------------------------------------------------------------------
Rearth = 6371000.0      # m
nm = 1852.0             # m
ft = 0.3048             # m
kts = 0.514444          # m/s
fpm = 0.00508           # m/s
g0 = 9.80665            # m/s2
R = 287.05287           # J/(kg K)
gamma = 1.40
p0 = 101325.0           # Pa
rho0 = 1.225            # kg/m3
T0 = 288.15             # K
Tstrat = 216.65         # K

# Frozen A320 envelope and autopilot defaults (docs/BLUESKY_SUBSET_SPEC.md §A.3).  The
# speed limit and the ground-phase envelope are FITTED to the reference's own SAC training
# logs (scripts/common/results/logs_backup/*_SAC.csv) by rolling out its saved actors
# (tests/golden/sac_actors.npz; tests/test_ref_logs.py):
#   VMAX_CAS: Descent + Vertical episode-length distributions (162.5..163.5 bracket)
#   VMAX_GD:  was fitted to Horizontal + PlanWaypoint episode lengths (88.5); round 5 pins it
#             at 89.0 from the saved models' observations (tests/test_last_obs.py)
# VSMAX is NOT fitted (round 4): the round-2 fit (12.1 m/s, from Descent SAC's final
# altitude) bound below the envs' 12.5 m/s command and the held-out DDPG / PPO actors
# rejected it; it is 4000 fpm, non-binding for every command the envs issue.
BANKDEF = math.radians(25.0)          # ap.bankdef
TAN_BANKDEF = 0.4663076581549986      # tan(BANKDEF), frozen literal shared with the device code
APVSDEF = 1500.0 * fpm                # ap.apvsdef  (m/s)
EPS_SPD = 0.01                        # traf.eps
AXMAX = 0.5                           # perf.axmax  (m/s2), airborne
VMIN_CAS = 140.0 * kts                # perf.vmin   (m/s CAS)
VMAX_CAS = 163.0                      # perf.vmax   (m/s CAS), fitted
MMO = 0.80                            # perf.mmo: the reference's saved Merge states hold the
                                      # ownship at M0.80 (tests/golden/extract_last_obs.py)
HMAX = 39800.0 * ft                   # perf.hmax   (m)
VSMAX = 4000.0 * fpm                  # perf.vsmax  (m/s), non-binding (the fit is withdrawn)
VSMIN = -4000.0 * fpm                 # perf.vsmin  (m/s); unreachable: the intent is |ap.vs|
GD_ALT_FT = 75.0                      # OpenAP phase GD: alt <= 75 ft
VMAX_GD = 89.0                        # perf.vmax in phase GD (m/s CAS); vmin 0.  Pinned by the
                                      # reference's saved HorizontalCR states: every aircraft at
                                      # TAS 89.000 at alt 0 (was fitted: 88.5)
AXMAX_GD = 2.0                        # perf.axmax in phase GD (m/s2)

# asas defaults (bluesky settings: asas_pzr, asas_pzh, asas_dtlookahead)
RPZ = 5.0 * nm
HPZ = 1000.0 * ft
DTLOOKAHEAD = 300.0


def pymod(a, b):
    """Python/NumPy floor-mod (``a % b`` with the sign of ``b``), elementwise."""
    return np.remainder(a, b)


def degto180(angle):
    """bluesky.tools.misc.degto180: (angle + 180) % 360 - 180."""
    return pymod(angle + 180.0, 360.0) - 180.0


# --------------------------------------------------------------------------------------
# aero  (bluesky/tools/aero.py: vatmos, vtas2cas, vcas2tas, vtas2mach, vmach2tas,
#        vcasormach2tas, vcasormach)
# --------------------------------------------------------------------------------------
def vatmos(h):
    T = np.maximum(288.15 - 0.0065 * h, Tstrat)
    rhotrop = 1.225 * (T / 288.15) ** 4.256848030018761
    dhstrat = np.maximum(0.0, h - 11000.0)
    rho = rhotrop * np.exp(-dhstrat / 6341.552161)
    p = rho * R * T
    return p, rho, T


def vtas2cas(tas, h):
    p, rho, T = vatmos(h)
    qdyn = p * ((1.0 + rho * tas * tas / (7.0 * p)) ** 3.5 - 1.0)
    cas = np.sqrt(7.0 * p0 / rho0 * ((qdyn / p0 + 1.0) ** (2.0 / 7.0) - 1.0))
    return np.where(tas < 0, -1 * cas, cas)


def vcas2tas(cas, h):
    p, rho, T = vatmos(h)
    qdyn = p0 * ((1.0 + rho0 * cas * cas / (7.0 * p0)) ** 3.5 - 1.0)
    tas = np.sqrt(7.0 * p / rho * ((1.0 + qdyn / p) ** (2.0 / 7.0) - 1.0))
    return np.where(cas < 0, -1 * tas, tas)


def vtas2mach(tas, h):
    p, rho, T = vatmos(h)
    a = np.sqrt(gamma * R * T)
    return tas / a


def vmach2tas(M, h):
    p, rho, T = vatmos(h)
    a = np.sqrt(gamma * R * T)
    return M * a


def vcasormach2tas(spd, h):
    return np.where(np.abs(spd) < 2.0, vmach2tas(spd, h), vcas2tas(spd, h))


def vcasormach(spd, h):
    ismach = np.logical_and(0.1 < spd, spd < 2.0)
    tas = np.where(ismach, vmach2tas(spd, h), vcas2tas(spd, h))
    cas = np.where(ismach, vtas2cas(tas, h), spd)
    m = np.where(ismach, spd, vtas2mach(tas, h))
    return tas, cas, m


# --------------------------------------------------------------------------------------
# geo  (bluesky/tools/geo.py)
# --------------------------------------------------------------------------------------
def kwikqdrdist(lata, lona, latb, lonb):
    """qdr [deg, 0..360), dist [NM].  Call sites: merge_env.py:179,181,203,280;
    vertical_cr_env.py:135,235."""
    re = 6371000.0
    dlat = np.radians(latb - lata)
    dlon = np.radians(pymod((lonb - lona) + 180, 360) - 180)
    cavelat = np.cos(np.radians(lata + latb) * 0.5)
    dangle = np.sqrt(dlat * dlat + dlon * dlon * cavelat * cavelat)
    dist = re * dangle / nm
    qdr = pymod(np.degrees(np.arctan2(dlon * cavelat, dlat)), 360.0)
    return qdr, dist


def kwikdist(lata, lona, latb, lonb):
    """dist [NM]. Call sites: vertical_cr_env.py:158, descent_env.py:102."""
    re = 6371000.0
    dlat = np.radians(latb - lata)
    dlon = np.radians(pymod((lonb - lona) + 180, 360) - 180)
    cavelat = np.cos(np.radians(lata + latb) * 0.5)
    dangle = np.sqrt(dlat * dlat + dlon * dlon * cavelat * cavelat)
    return re * dangle / nm


def kwikdist_matrix(lata, lona, latb, lonb):
    """dist [NM] with the matrix-form operation order
    ``sqrt(dlat*dlat + (dlon*dlon)*(cavelat*cavelat))`` (call site merge_env.py:195).
    Elementwise on broadcast-compatible inputs."""
    re = 6371000.0
    dlat = np.radians(latb - lata)
    dlon = np.radians(pymod((lonb - lona) + 180, 360) - 180)
    cavelat = np.cos(np.radians(latb + lata) * 0.5)
    dangle = np.sqrt(np.multiply(dlat, dlat) +
                     np.multiply(np.multiply(dlon, dlon), np.multiply(cavelat, cavelat)))
    return re * dangle / nm


def kwikqdrdist_matrix(lata, lona, latb, lonb):
    """Matrix form used by StateBased.detect; [.., i, j] = from a_i to b_j when called
    with lata[..., :, None] and latb[..., None, :]."""
    re = 6371000.0
    dlat = np.radians(latb - lata)
    dlon = np.radians(pymod((lonb - lona) + 180, 360) - 180)
    cavelat = np.cos(np.radians(lata + latb) * 0.5)
    dangle = np.sqrt(np.multiply(dlat, dlat) +
                     np.multiply(np.multiply(dlon, dlon), np.multiply(cavelat, cavelat)))
    dist = re * dangle / nm
    qdr = pymod(np.degrees(np.arctan2(np.multiply(dlon, cavelat), dlat)), 360.0)
    return qdr, dist


def kwikpos(latd1, lond1, qdr, dist):
    """Flat-earth destination (used by Traffic.creconfs)."""
    dx = dist * np.sin(np.radians(qdr))
    dy = dist * np.cos(np.radians(qdr))
    dlat = dy / 60.0
    dlon = dx / (np.maximum(0.01, 60.0 * np.cos(np.radians(latd1))))
    latd2 = latd1 + dlat
    lond2 = pymod((lond1 + dlon) + 180, 360) - 180
    return latd2, lond2


def rwgs84(latd):
    lat = np.radians(latd)
    a = 6378137.0
    b = 6356752.314245
    coslat = np.cos(lat)
    sinlat = np.sin(lat)
    an = a * a * coslat
    bn = b * b * sinlat
    ad = a * coslat
    bd = b * sinlat
    return np.sqrt((an * an + bn * bn) / (ad * ad + bd * bd))


def qdrdist(latd1, lond1, latd2, lond2):
    """WGS84 bearing [deg, -180..180] and distance [NM] (LNAV guidance)."""
    res1 = rwgs84(0.5 * (latd1 + latd2))
    a = 6378137.0
    r1 = rwgs84(latd1)
    r2 = rwgs84(latd2)
    res2 = 0.5 * (np.abs(latd1) * (r1 + a) + np.abs(latd2) * (r2 + a)) / \
        (np.maximum(0.000001, np.abs(latd1) + np.abs(latd2)))
    sw = (latd1 * latd2 >= 0.0)
    r = np.where(sw, res1, res2)
    lat1 = np.radians(latd1)
    lon1 = np.radians(lond1)
    lat2 = np.radians(latd2)
    lon2 = np.radians(lond2)
    d = r * np.arccos(np.cos(lat1) * np.cos(lat2) * np.cos(lon2 - lon1) +
                      np.sin(lat1) * np.sin(lat2))
    coslat1 = np.cos(lat1)
    coslat2 = np.cos(lat2)
    qdr = np.degrees(np.arctan2(np.sin(lon2 - lon1) * coslat2,
                                coslat1 * np.sin(lat2) -
                                np.sin(lat1) * coslat2 * np.cos(lon2 - lon1)))
    return qdr, d / nm


# --------------------------------------------------------------------------------------
# Traffic state (SoA, any leading shape) and Traffic.update
# --------------------------------------------------------------------------------------
FIELDS_F64 = ("lat", "lon", "alt", "hdg", "trk", "tas", "cas", "gs", "vs",
              "gsnorth", "gseast", "ax",
              "ap_trk", "selspd", "selalt", "selvs")
FIELDS_I32 = ("swlnav", "actwp")


class TrafState:
    """Structure-of-arrays aircraft state.  ``actwp`` indexes the env-kind route table
    (``route_lat/route_lon``: waypoint k of the shared route); ``swlnav`` is LNAV on."""

    def __init__(self, shape):
        for f in FIELDS_F64:
            setattr(self, f, np.zeros(shape, np.float64))
        self.swlnav = np.zeros(shape, bool)
        self.actwp = np.zeros(shape, np.int32)

    def copy(self):
        out = TrafState(self.lat.shape)
        for f in FIELDS_F64:
            setattr(out, f, getattr(self, f).copy())
        out.swlnav = self.swlnav.copy()
        out.actwp = self.actwp.copy()
        return out


def cre_state(st, idx, aclat, aclon, achdg, acalt, acspd):
    """Traffic.cre: position, heading, speed (acspd is CAS [m/s] or Mach),
    autopilot initialised to hold the creation state."""
    tas, cas, _m = vcasormach(np.asarray(acspd, np.float64), np.asarray(acalt, np.float64))
    st.lat[idx] = aclat
    st.lon[idx] = aclon
    st.alt[idx] = acalt
    st.hdg[idx] = achdg
    st.trk[idx] = achdg
    st.tas[idx] = tas
    st.cas[idx] = cas
    st.gs[idx] = tas
    hdgrad = np.radians(achdg)
    st.gsnorth[idx] = tas * np.cos(hdgrad)
    st.gseast[idx] = tas * np.sin(hdgrad)
    st.vs[idx] = 0.0
    st.ax[idx] = 0.0
    st.ap_trk[idx] = achdg          # autopilot.create: ap.trk = traf.trk
    st.selspd[idx] = cas            # traffic.cre: selspd = cas
    st.selalt[idx] = acalt          # traffic.cre: selalt = alt
    st.selvs[idx] = 0.0
    st.swlnav[idx] = False
    st.actwp[idx] = 0


def ground_phase(alt):
    """OpenAP flight phase GD (bluesky performance/openap/phase.py): alt <= 75 ft."""
    return alt / ft <= GD_ALT_FT


def perf_limits(intent_tas, intent_vs, intent_h, ax, ground=False):
    """OpenAP-style PerfModel.limits with the frozen A320 envelope; `ground` = phase GD
    (its own speed envelope and axmax)."""
    vmin = np.where(ground, 0.0, VMIN_CAS)
    vmax = np.where(ground, VMAX_GD, VMAX_CAS)
    axmax = np.where(ground, AXMAX_GD, AXMAX)
    allow_h = np.where(intent_h > HMAX, HMAX, intent_h)
    intent_cas = vtas2cas(intent_tas, allow_h)
    allow_cas = np.where(intent_cas < vmin, vmin, intent_cas)
    allow_cas = np.where(intent_cas > vmax, vmax, allow_cas)
    allow_tas = vcas2tas(allow_cas, allow_h)
    allow_tas = np.where(vtas2mach(allow_tas, allow_h) > MMO, vmach2tas(MMO, allow_h), allow_tas)
    vs_max_with_acc = (1 - ax / axmax) * VSMAX
    allow_vs = np.where((intent_vs > 0) & (intent_vs > VSMAX), vs_max_with_acc, intent_vs)
    allow_vs = np.where((intent_vs < 0) & (intent_vs < VSMIN), VSMIN, allow_vs)
    return allow_tas, allow_vs, allow_h


# --------------------------------------------------------------------------------------
# Wind field (bluesky.traffic.windfield.Windfield; used by bluesky_gym/wrappers/wind.py:26)
# Frozen definition (docs/BLUESKY_SUBSET_SPEC.md §A.7): profiles live on a fixed altitude
# axis 0..45000 ft in 100 ft steps; horizontal interpolation is inverse-distance-squared
# weighting, summed in point order.
# --------------------------------------------------------------------------------------
WIND_ALTSTEP = 100.0 * ft
WIND_ALTMAX = 45000.0 * ft
WIND_NALT = 451
WIND_ALTAXIS = np.arange(WIND_NALT, dtype=np.float64) * WIND_ALTSTEP


class WindField:
    def __init__(self):
        self.clear()

    def clear(self):
        self.lat = np.zeros(0)
        self.lon = np.zeros(0)
        self.vnorth = np.zeros((1, 0))      # [levels][P]; levels = 1 (2-D) or WIND_NALT
        self.veast = np.zeros((1, 0))
        self.winddim = 0

    def addpointvne(self, lat, lon, vnorth, veast, windalt=None):
        """Add P points.  vnorth/veast: [P] or [1, P] (constant in altitude) or
        [len(windalt), P] profiles over windalt (interpolated onto the fixed axis)."""
        lat = np.atleast_1d(np.asarray(lat, np.float64)).ravel()
        lon = np.atleast_1d(np.asarray(lon, np.float64)).ravel()
        P = lat.size
        vn = np.asarray(vnorth, np.float64)
        ve = np.asarray(veast, np.float64)
        if windalt is None:
            vn = vn.reshape(-1)[-P:].reshape(1, P) if vn.size != P else vn.reshape(1, P)
            ve = ve.reshape(-1)[-P:].reshape(1, P) if ve.size != P else ve.reshape(1, P)
            prof3d = False
        else:
            wa = np.atleast_1d(np.asarray(windalt, np.float64))
            vn = vn.reshape(len(wa), P)
            ve = ve.reshape(len(wa), P)
            vn = np.stack([np.interp(WIND_ALTAXIS, wa, vn[:, p]) for p in range(P)], 1)
            ve = np.stack([np.interp(WIND_ALTAXIS, wa, ve[:, p]) for p in range(P)], 1)
            prof3d = True
        if self.winddim == 3 or prof3d:
            # bring every table to the full axis
            def full(t):
                return t if t.shape[0] == WIND_NALT else np.repeat(t[:1], WIND_NALT, 0)
            self.vnorth = np.concatenate([full(self.vnorth), full(vn)], 1)
            self.veast = np.concatenate([full(self.veast), full(ve)], 1)
        else:
            self.vnorth = np.concatenate([self.vnorth, vn], 1)
            self.veast = np.concatenate([self.veast, ve], 1)
        self.lat = np.concatenate([self.lat, lat])
        self.lon = np.concatenate([self.lon, lon])
        self.winddim = 3 if (prof3d or self.winddim == 3) else min(2, self.lat.size)
        return self.lat.size - 1

    def getdata(self, lat, lon, alt):
        lat = np.asarray(lat, np.float64)
        lon = np.asarray(lon, np.float64)
        alt = np.asarray(alt, np.float64)
        shape = np.broadcast(lat, lon, alt).shape
        if self.winddim == 0:
            return np.zeros(shape), np.zeros(shape)
        if self.winddim == 1:
            return np.full(shape, self.vnorth[0, 0]), np.full(shape, self.veast[0, 0])
        P = self.lat.size
        w = []
        S = np.zeros(shape)
        for p in range(P):
            cavelat = np.cos(np.radians(0.5 * (lat + self.lat[p])))
            dy = np.radians(lat - self.lat[p])
            dx = cavelat * np.radians(lon - self.lon[p])
            wp = 1.0 / (1e-16 + dx * dx + dy * dy)
            w.append(wp)
            S = S + wp
        if self.winddim == 3:
            idx = np.minimum(np.maximum(alt, 0.0), WIND_ALTMAX) / WIND_ALTSTEP
            ialt = np.minimum(np.floor(idx).astype(np.int64), WIND_NALT - 2)
            falt = idx - ialt
        vn = np.zeros(shape)
        ve = np.zeros(shape)
        for p in range(P):
            h = w[p] / S
            if self.winddim == 3:
                cn = (1.0 - falt) * self.vnorth[ialt, p] + falt * self.vnorth[ialt + 1, p]
                ce = (1.0 - falt) * self.veast[ialt, p] + falt * self.veast[ialt + 1, p]
            else:
                cn, ce = self.vnorth[0, p], self.veast[0, p]
            vn = vn + cn * h
            ve = ve + ce * h
        return vn, ve

    def table(self):
        """(lat[P], lon[P], vnorth[levels][P], veast[levels][P]) for the device."""
        return self.lat.copy(), self.lon.copy(), self.vnorth.copy(), self.veast.copy()


def wind_active(wind):
    return wind is not None and wind.winddim > 0


def selhdg_track(st, idx, hdg, wind):
    """Autopilot.selhdgcmd: the commanded heading becomes a track through the wind
    triangle at the current position when airborne (alt > 50 ft)."""
    hdg = np.asarray(hdg, np.float64)
    if not wind_active(wind):
        return hdg
    alt, tas = st.alt[idx], st.tas[idx]
    vn, ve = wind.getdata(st.lat[idx], st.lon[idx], alt)
    tasnorth = tas * np.cos(np.radians(hdg))
    taseast = tas * np.sin(np.radians(hdg))
    trk = np.degrees(np.arctan2(taseast + ve, tasnorth + vn)) % 360.0
    return np.where(alt > 50.0 * ft, trk, hdg)


def wind_obs(st, wind, max_wind=50.0):
    """bluesky_gym/wrappers/wind.py:56-66 (_get_wind_observation), ownship = index 0."""
    lat, lon, alt = st.lat[..., 0], st.lon[..., 0], st.alt[..., 0]
    wn, we = wind.getdata(lat, lon, alt)
    hdg = np.deg2rad(st.hdg[..., 0])
    wind_u = (wn * np.cos(hdg) + we * np.sin(hdg)) / max_wind
    wind_v = (-wn * np.sin(hdg) + we * np.cos(hdg)) / max_wind
    return wind_u, wind_v


def traffic_update(st, dt, route_lat, route_lon, route_next_qdr, wind=None):
    """One simulation substep (Traffic.update, ASAS resolution off).

    route_lat/route_lon: 1-D arrays of the shared route's waypoints (may be empty).
    route_next_qdr[k]: bearing from waypoint k to waypoint k+1 (-999 for the last).
    wind: WindField or None.
    """
    windy = wind_active(wind)
    if windy:
        vwn, vwe = wind.getdata(st.lat, st.lon, st.alt)
    nwp = len(route_lat)
    # ---- autopilot (Autopilot.update) --------------------------------------------
    if nwp > 0:
        lnav = st.swlnav
        wlat = np.asarray(route_lat)[np.clip(st.actwp, 0, nwp - 1)]
        wlon = np.asarray(route_lon)[np.clip(st.actwp, 0, nwp - 1)]
        qdr, distnm = qdrdist(st.lat, st.lon, wlat, wlon)
        dist = distnm * nm
        # ActiveWaypoint.reached: fly-by turn distance, or "too close and passing"
        nq = np.asarray(route_next_qdr)[np.clip(st.actwp, 0, nwp - 1)]
        next_qdr = np.where(nq < -900.0, qdr, nq)
        turnrad = st.tas * st.tas / (np.maximum(0.01, TAN_BANKDEF) * g0)
        turndist = np.abs(turnrad * np.tan(np.radians(
            0.5 * np.abs(degto180(pymod(qdr, 360.0) - pymod(next_qdr, 360.0))))))
        close2wp = dist / (np.maximum(0.0001, np.abs(st.gs))) < 4.0
        tooclose2turn = close2wp & (np.abs(degto180(pymod(st.trk, 360.0) - pymod(qdr, 360.0))) > 90.0)
        reached = lnav & ((dist < turndist) | tooclose2turn)
        last = st.actwp >= nwp - 1
        # last waypoint reached: LNAV off, keep commanded track
        st.swlnav = np.where(reached & last, False, st.swlnav)
        adv = reached & ~last
        if adv.any():
            st.actwp = np.where(adv, st.actwp + 1, st.actwp)
            wlat2 = np.asarray(route_lat)[np.clip(st.actwp, 0, nwp - 1)]
            wlon2 = np.asarray(route_lon)[np.clip(st.actwp, 0, nwp - 1)]
            qdr2, _ = qdrdist(st.lat, st.lon, wlat2, wlon2)
            qdr = np.where(adv, qdr2, qdr)
        st.ap_trk = np.where(st.swlnav, qdr, st.ap_trk)
    ap_vs = np.where(np.abs(st.selvs) > 0.1, st.selvs, APVSDEF)
    ap_alt = st.selalt
    ap_tas = vcasormach2tas(st.selspd, st.alt)
    # ---- aporasas (no active resolution) ------------------------------------------
    trk_cmd = st.ap_trk
    vs_cmd = np.abs(ap_vs)
    if windy:
        # ActivePilot: heading that flies the commanded track through the wind
        Vw = np.sqrt(vwn * vwn + vwe * vwe)
        winddir = np.arctan2(vwe, vwn)
        drift = np.radians(trk_cmd) - winddir
        steer = np.arcsin(np.minimum(1.0, np.maximum(-1.0, Vw * np.sin(drift) /
                                                     np.maximum(0.001, st.tas))))
        hdg_cmd = pymod(trk_cmd + np.degrees(steer), 360.0)
    else:
        hdg_cmd = pymod(trk_cmd, 360.0)
    # ---- performance limits ------------------------------------------------------------
    ground = ground_phase(st.alt)
    tas_cmd, vs_cmd, alt_cmd = perf_limits(ap_tas, vs_cmd, ap_alt, st.ax, ground)
    # ---- update_airspeed ------------------------------------------------------------
    axmax = np.where(ground, AXMAX_GD, AXMAX)
    delta_spd = tas_cmd - st.tas
    need_ax = np.abs(delta_spd) > np.abs(dt * axmax)
    st.ax = need_ax * np.sign(delta_spd) * axmax
    st.tas = np.where(need_ax, st.tas + st.ax * dt, tas_cmd)
    st.cas = vtas2cas(st.tas, st.alt)
    turnrate = np.degrees(g0 * TAN_BANKDEF / np.maximum(st.tas, EPS_SPD))
    delhdg = pymod(hdg_cmd - st.hdg + 180.0, 360.0) - 180.0
    swhdgsel = np.abs(delhdg) > np.abs(dt * turnrate)
    st.hdg = pymod(np.where(swhdgsel, st.hdg + dt * turnrate * np.sign(delhdg), hdg_cmd), 360.0)
    delta_alt = alt_cmd - st.alt
    swaltsel = np.abs(delta_alt) > np.maximum(10 * ft, np.abs(2 * np.abs(dt * st.vs)))
    target_vs = swaltsel * np.sign(delta_alt) * np.abs(vs_cmd)
    delta_vs = target_vs - st.vs
    need_az = np.abs(delta_vs) > 300 * fpm
    az = need_az * np.sign(delta_vs) * (300 * fpm)
    st.vs = np.where(need_az, st.vs + az * dt, target_vs)
    st.vs = np.where(np.isfinite(st.vs), st.vs, 0)
    # ---- update_groundspeed ------------------------------------------------------------
    if windy:
        applywind = st.alt > 50.0 * ft
        st.gsnorth = st.tas * np.cos(np.radians(st.hdg)) + vwn * applywind
        st.gseast = st.tas * np.sin(np.radians(st.hdg)) + vwe * applywind
        st.gs = np.where(applywind, np.sqrt(st.gsnorth * st.gsnorth + st.gseast * st.gseast),
                         st.tas)
        st.trk = np.where(applywind, pymod(np.degrees(np.arctan2(st.gseast, st.gsnorth)), 360.0),
                          st.hdg)
    else:
        st.gsnorth = st.tas * np.cos(np.radians(st.hdg))
        st.gseast = st.tas * np.sin(np.radians(st.hdg))
        st.gs = st.tas.copy()
        st.trk = st.hdg.copy()
    # ---- update_pos -------------------------------------------------------------------
    st.alt = np.where(swaltsel, np.round(st.alt + st.vs * dt, 6), alt_cmd)
    st.lat = st.lat + np.degrees(dt * st.gsnorth / Rearth)
    coslat = np.cos(np.deg2rad(st.lat))
    st.lon = st.lon + np.degrees(dt * st.gseast / coslat / Rearth)


# --------------------------------------------------------------------------------------
# StateBased conflict detection (bluesky/traffic/asas/statebased.py: detect)
# --------------------------------------------------------------------------------------
def statebased_detect(lat, lon, alt, trk, gs, vs, rpz=RPZ, hpz=HPZ, dtlookahead=DTLOOKAHEAD,
                      active=None):
    """All-pairs CPA over the last axis (N aircraft).  Returns a dict with
    swconfl[..., i, j], swlos[..., i, j], inconf[..., i], tcpamax[..., i],
    dist (m), tcpa, dcpa2, tinconf, toutconf.  [i, j] = aircraft j relative to i.
    active[..., N] (optional): aircraft that exist (SectorCR's per-episode count); pairs
    with an absent aircraft are neither conflicts, LoS nor part of min_sep."""
    n = lat.shape[-1]
    eye = np.eye(n, dtype=bool)
    I = eye.astype(np.float64)
    qdr, dist = kwikqdrdist_matrix(lat[..., :, None], lon[..., :, None],
                                   lat[..., None, :], lon[..., None, :])
    dist = dist * nm + 1e9 * I
    qdrrad = np.radians(qdr)
    dx = dist * np.sin(qdrrad)
    dy = dist * np.cos(qdrrad)
    trkrad = np.radians(trk)
    u = gs * np.sin(trkrad)
    v = gs * np.cos(trkrad)
    du = u[..., None, :] - u[..., :, None]
    dv = v[..., None, :] - v[..., :, None]
    dv2 = du * du + dv * dv
    dv2 = np.where(np.abs(dv2) < 1e-6, 1e-6, dv2)
    vrel = np.sqrt(dv2)
    tcpa = -(du * dx + dv * dy) / dv2 + 1e9 * I
    dcpa2 = np.abs(dist * dist - tcpa * tcpa * dv2)
    R2 = rpz * rpz
    swhorconf = dcpa2 < R2
    dxinhor = np.sqrt(np.maximum(0.0, R2 - dcpa2))
    dtinhor = dxinhor / vrel
    tinhor = np.where(swhorconf, tcpa - dtinhor, 1e8)
    touthor = np.where(swhorconf, tcpa + dtinhor, -1e8)
    dalt = alt[..., None, :] - alt[..., :, None] + 1e9 * I
    dvs = vs[..., None, :] - vs[..., :, None]
    dvs = np.where(np.abs(dvs) < 1e-6, 1e-6, dvs)
    tcrosshi = (dalt + hpz) / -dvs
    tcrosslo = (dalt - hpz) / -dvs
    tinver = np.minimum(tcrosshi, tcrosslo)
    toutver = np.maximum(tcrosshi, tcrosslo)
    tinconf = np.maximum(tinver, tinhor)
    toutconf = np.minimum(toutver, touthor)
    swconfl = swhorconf & (tinconf <= toutconf) & (toutconf > 0.0) & \
        (tinconf < dtlookahead) & ~eye
    swlos = (dist < rpz) & (np.abs(dalt) < hpz)
    if active is not None:
        pair = active[..., :, None] & active[..., None, :]
        swconfl = swconfl & pair
        swlos = swlos & pair
        eye = eye | ~pair
    inconf = np.any(swconfl, -1)
    tcpamax = np.max(tcpa * swconfl, -1)
    # minimum separation among the pairs inside the StateBased horizon (the pairs whose
    # conflict state can be true): dist <= (RPZ + DTLOOKAHEAD*vrel)(1+1e-9) + 1 m
    horizon = (rpz + dtlookahead * vrel) * (1.0 + 1e-9) + 1.0
    inside = (dist <= horizon) & ~eye
    min_sep = np.min(np.where(inside, dist, np.inf), axis=(-2, -1))
    return dict(swconfl=swconfl, swlos=swlos, inconf=inconf, tcpamax=tcpamax,
                dist=dist, tcpa=tcpa, dcpa2=dcpa2, tinconf=tinconf, toutconf=toutconf,
                vrel=vrel, min_sep=min_sep)


# --------------------------------------------------------------------------------------
# creconfs (bluesky/traffic/traffic.py: Traffic.creconfs) -- scalar, Python math
# --------------------------------------------------------------------------------------
def creconfs_params(latref, lonref, altref, trkref_deg, gsref, vsref,
                    dpsi, dcpa, tlosh, dH=None, tlosv=None):
    """Returns (aclat, aclon, achdg, acalt, acspd_cas, acvs) of an intruder placed in
    conflict with the reference aircraft (spd=None branch: same ground speed)."""
    trkref = math.radians(trkref_deg)
    cpa = dcpa * nm
    pzr = RPZ
    pzh = HPZ
    trk = trkref + math.radians(dpsi)
    if dH is None:
        acalt = altref
        acvs = 0.0
    else:
        acalt = altref + dH
        tlosv = tlosh if tlosv is None else tlosv
        acvs = vsref - np.sign(dH) * (abs(dH) - pzh) / tlosv
    gsn, gse = gsref * math.cos(trk), gsref * math.sin(trk)
    vreln, vrele = gsref * math.cos(trkref) - gsn, gsref * math.sin(trkref) - gse
    vrel = math.sqrt(vreln * vreln + vrele * vrele)
    drelcpa = tlosh * vrel + (0 if cpa > pzr else math.sqrt(pzr * pzr - cpa * cpa))
    dist = math.sqrt(drelcpa * drelcpa + cpa * cpa)
    rd = drelcpa / dist
    rx = cpa / dist
    brn = math.degrees(math.atan2(-rx * vreln + rd * vrele, rd * vreln + rx * vrele))
    aclat, aclon = kwikpos(latref, lonref, brn, dist / nm)
    tasn, tase = gsn, gse
    acspd = vtas2cas(math.sqrt(tasn * tasn + tase * tase), acalt)
    achdg = math.degrees(math.atan2(tase, tasn))
    return (float(aclat), float(aclon), float(achdg), float(acalt), float(acspd), float(acvs))


# --------------------------------------------------------------------------------------
# get_point_at_distance (bluesky_gym/envs/common/functions.py:24-42)
# bound_angle_positive_negative_180 (functions.py:4-22)
# --------------------------------------------------------------------------------------
def get_point_at_distance(lat1, lon1, d, bearing, R=6371):
    lat1 = np.radians(lat1)
    lon1 = np.radians(lon1)
    a = np.radians(bearing)
    lat2 = np.arcsin(np.sin(lat1) * np.cos(d / R) + np.cos(lat1) * np.sin(d / R) * np.cos(a))
    lon2 = lon1 + np.arctan2(np.sin(a) * np.sin(d / R) * np.cos(lat1),
                             np.cos(d / R) - np.sin(lat1) * np.sin(lat2))
    return np.degrees(lat2), np.degrees(lon2)


def bound_angle_positive_negative_180(angle_deg):
    """Single wrap only (functions.py:17-22), elementwise."""
    a = np.asarray(angle_deg, np.float64)
    return np.where(a > 180, -(360 - a), np.where(a < -180, 360 + a, a))
