"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- polygons of SectorCREnv-v0 / StaticObstacleEnv-v0.

Restates
* ``bluesky_gym/envs/common/functions.py``: random_point_on_circle (:44-59, here from the
  uniform draw u), sort_points_clockwise (:61-75), polygon_area (:77-96), nm_to_latlong
  (:98-114), latlong_to_nm (:116-132), euclidean_distance (:134-148), get_hdg (:150-175);
* ``bluesky.tools.areafilter`` POLY areas (``defineArea``/``checkInside``, call sites
  sector_cr_env.py:134-139,158,197 and static_obstacle_env.py:181,205,329-338): the border
  is a matplotlib ``Path`` over (lat, lon) vertices and ``contains_points`` is the even-odd
  crossing test of ``point_in_path`` (Haines): edge (v0 -> v1) toggles the state of point
  (tx, ty) when ``(v0.y >= ty) != (v1.y >= ty)`` and
  ``((v1.y - ty) * (v0.x - v1.x) >= (v1.x - tx) * (v0.y - v1.y)) == (v1.y >= ty)``,
  with x = lat, y = lon, over the closed vertex ring.  Frozen in
  docs/BLUESKY_SUBSET_SPEC.md §A.8 (bluesky-simulator is absent: parity unpinned at this
  layer; the env layer on top is pinned by the golden vectors).

Also the device-side (Philox) scenario generators of the two envs, restated draw for draw
from bsg_kernels.hip so that batch parity tests can reproduce device resets.
"""
from __future__ import annotations

import numpy as np

from . import bluesky_subset as bsx
from . import philox

# --------------------------------------------------------------------------------------
# functions.py
# --------------------------------------------------------------------------------------


def point_on_circle(radius, u):
    """random_point_on_circle with the np.random.uniform(0, 1) draw u."""
    alpha = 2 * np.pi * u
    return np.array([radius * np.cos(alpha), radius * np.sin(alpha)])


def sort_points_clockwise(vertices):
    return [vertices[i] for i in np.argsort([np.arctan2(v[1], v[0]) for v in vertices])]


def polygon_area(vertices):
    n = len(vertices)
    area = 0.0
    for i in range(n):
        x1, y1 = vertices[i]
        x2, y2 = vertices[(i + 1) % n]
        area += x1 * y2 - y1 * x2
    return np.abs(area) / 2.0


def nm_to_latlong(center, point):
    lat = center[0] + (point[0] / 60)
    lon = center[1] + (point[1] / (60 * np.cos(np.radians(center[0]))))
    return np.array([lat, lon])


def latlong_to_nm(center, point):
    x = (point[0] - center[0]) * 60
    y = (point[1] - center[1]) * 60 * np.cos(np.radians(center[0]))
    return np.array([x, y])


def euclidean_distance(p1, p2):
    return np.sqrt(np.sum((p2 - p1) ** 2))


def get_hdg(point1, point2):
    lat1, lon1 = np.radians(point1)
    lat2, lon2 = np.radians(point2)
    delta_lon = lon2 - lon1
    x = np.sin(delta_lon) * np.cos(lat2)
    y = np.cos(lat1) * np.sin(lat2) - np.sin(lat1) * np.cos(lat2) * np.cos(delta_lon)
    hdg = np.degrees(np.arctan2(x, y))
    return (hdg + 360) % 360


# --------------------------------------------------------------------------------------
# areafilter POLY containment
# --------------------------------------------------------------------------------------
def points_in_poly(lat, lon, plat, plon):
    """Even-odd crossing test of (lat, lon) against the closed ring (plat[k], plon[k])."""
    tx = np.asarray(lat, np.float64)
    ty = np.asarray(lon, np.float64)
    inside = np.zeros(np.broadcast(tx, ty).shape, bool)
    n = len(plat)
    for k in range(n):
        x0, y0 = plat[k], plon[k]
        x1, y1 = plat[(k + 1) % n], plon[(k + 1) % n]
        yflag0 = y0 >= ty
        yflag1 = y1 >= ty
        cross = (yflag0 != yflag1) & ((((y1 - ty) * (x0 - x1)) >= ((x1 - tx) * (y0 - y1))) == yflag1)
        inside ^= cross
    return inside


class AreaFilter:
    """bluesky.tools.areafilter subset: named POLY areas (top/bottom +-1e9)."""

    def __init__(self):
        self.areas = {}

    def defineArea(self, name, shape, coordinates, top=1e9, bottom=-1e9):
        assert shape.upper() == "POLY"
        c = np.asarray(coordinates, np.float64).reshape(-1, 2)
        self.areas[name] = (c[:, 0].copy(), c[:, 1].copy(), top, bottom)
        return True

    def deleteArea(self, name):
        self.areas.pop(name, None)

    def checkInside(self, name, lat, lon, alt):
        plat, plon, top, bottom = self.areas[name]
        ins = points_in_poly(lat, lon, plat, plon)
        alt = np.asarray(alt, np.float64)
        return ins & (bottom <= alt) & (alt <= top)


# --------------------------------------------------------------------------------------
# polygon generation (sector_cr_env.py:140-158, static_obstacle_env.py:148-162)
# --------------------------------------------------------------------------------------
def build_polygon(R, us, min_area):
    """Polygon from the uniform draws us (consumed until the area reaches min_area).
    Returns (points NM sorted as the reference keeps them, area, number of draws used)."""
    p = [point_on_circle(R, us[k]) for k in range(3)]
    p = sort_points_clockwise(p)
    a = polygon_area(p)
    k = 3
    while a < min_area and k < len(us):
        p.append(point_on_circle(R, us[k]))
        p = sort_points_clockwise(p)
        a = polygon_area(p)
        k += 1
    return p, a, k


STATIC_NUM_OBSTACLES = 10
STATIC_VMAX = 16                 # vertices kept per obstacle polygon (device layout)
SECTOR_VMAX = 32                 # sector polygon vertices (device layout)
SECTOR_CENTER = np.array([51.990426702297746, 4.376124857109851])
SECTOR_POLY_AREA_RANGE = (2400, 3750)
OBSTACLE_AREA_RANGE = (50, 1000)
TAG_STAT = 0x53544154            # 'STAT'
TAG_SECT = 0x53454354            # 'SECT'


def _u01(x, y):
    return float(philox.u01_53(np.uint32(x), np.uint32(y)))


def _ph(env, ep, draw, tag, seed):
    r = philox.philox4x32_10(np.uint32(env), np.uint32(ep), np.uint32(draw), np.uint32(tag), seed)
    return [int(v) for v in r]


def _randint(x, lo, hi):
    return int(philox.randint_u32(np.uint32(x), lo, hi))


def static_device_spawn(env, ep, seed):
    """Draws of the device StaticObstacle reset (bsg_kernels.hip spawn_static): the host
    spawn-parameter row [per obstacle: dis, hdg, area, nvert, u[16]] + [wdis, whdg]."""
    row = []
    cen = []
    for o in range(STATIC_NUM_OBSTACLES):
        x, y, z, _ = _ph(env, ep, o, TAG_STAT, seed)
        dis, hdg, area = _randint(x, 20, 150), _randint(y, 0, 360), _randint(z, 100, 1000)
        us = []
        for k in range(STATIC_VMAX):
            a, b, _, _ = _ph(env, ep, 16 + o * STATIC_VMAX + k, TAG_STAT, seed)
            us.append(_u01(a, b))
        R = np.sqrt(area / np.pi)
        _, _, nv = build_polygon(R, us, OBSTACLE_AREA_RANGE[0])
        row += [dis, hdg, area, nv] + us
        cen.append((dis, hdg, area, nv, us))
    polys = static_polygons(np.array(row + [0.0, 0.0]))
    wd = wh = 0
    for t in range(1000):
        x, y, _, _ = _ph(env, ep, 1000 + t, TAG_STAT, seed)
        wd, wh = _randint(x, 100, 170), _randint(y, 0, 360)
        wlat, wlon = bsx.get_point_at_distance(52.0, 4.0, wd, wh)
        if not any(points_in_poly(wlat, wlon, pl[0], pl[1]) for pl in polys["poly"]):
            break
    return np.array(row + [wd, wh], np.float64)


def static_polygons(row):
    """Obstacle geometry from a spawn row: centres, radii, (lat, lon) vertex rings, and the
    waypoint (static_obstacle_env.py:163-228)."""
    cl, cn, rr, polys = [], [], [], []
    W = 4 + STATIC_VMAX
    for o in range(STATIC_NUM_OBSTACLES):
        dis, hdg, area, nv = row[o * W: o * W + 4]
        us = row[o * W + 4: (o + 1) * W]
        clat, clon = bsx.get_point_at_distance(52.0, 4.0, dis, hdg)
        R = np.sqrt(int(area) / np.pi)
        p = [point_on_circle(R, us[k]) for k in range(3)]
        p = sort_points_clockwise(p)
        for k in range(3, int(nv)):
            p.append(point_on_circle(R, us[k]))
            p = sort_points_clockwise(p)
        ll = [nm_to_latlong((clat, clon), q) for q in p]
        polys.append((np.array([q[0] for q in ll]), np.array([q[1] for q in ll])))
        cl.append(clat); cn.append(clon); rr.append(R)
    wd, wh = row[STATIC_NUM_OBSTACLES * W: STATIC_NUM_OBSTACLES * W + 2]
    wlat, wlon = bsx.get_point_at_distance(52.0, 4.0, wd, wh)
    return {"clat": np.array(cl), "clon": np.array(cn), "R": np.array(rr), "poly": polys,
            "wpt": (float(wlat), float(wlon))}


def sector_build(R_area_max, us, min_area):
    R = np.sqrt(R_area_max / np.pi)
    return build_polygon(R, us, min_area)


def sector_device_spawn(env, ep, seed, N, density_mode="normal"):
    """Draws of the device SectorCR reset (bsg_kernels.hip sector_plan): returns the host
    spawn-parameter row [nac, nvert, plat[32], plon[32], wlat, wlon, (lat, lon, hdg) x N]."""
    us = []
    for k in range(SECTOR_VMAX):
        a, b, _, _ = _ph(env, ep, k, TAG_SECT, seed)
        us.append(_u01(a, b))
    p, area, nv = sector_build(SECTOR_POLY_AREA_RANGE[1], us, SECTOR_POLY_AREA_RANGE[0])
    x, y, z, w = _ph(env, ep, 64, TAG_SECT, seed)
    if density_mode == "normal":
        u1 = 1.0 - _u01(x, y)
        u2 = _u01(z, w)
        zn = np.sqrt(-2.0 * np.log(u1)) * np.cos(2 * np.pi * u2)
        dens = 0.005 + 0.001 * zn
    else:
        dens = 0.003 + (0.007 - 0.003) * _u01(x, y)
    nac = int(max(np.ceil(dens * area), 4 + 1))
    nac = min(nac, N)
    ds = []
    for i in range(nac):
        a, b, _, _ = _ph(env, ep, 128 + i, TAG_SECT, seed)
        ds.append(_u01(a, b))
    return _sector_row(p, area, nac, ds, N, lambda i, t: _ph(env, ep, 0x10000 + i * 4096 + t,
                                                              TAG_SECT, seed))


def sector_waypoints(p, d_units):
    """sector_cr_env.py:160-182 with the draws d = uniform(0, perim) = perim * u."""
    perim = 0
    for i in range(len(p)):
        perim += euclidean_distance(np.array(p[i]), np.array(p[(i + 1) % len(p)]))
    return _sector_wpts_from_d(p, [0.0 + (perim - 0.0) * u for u in d_units])


def _sector_row(p, area, nac, d_units, N, draw):
    pts = np.array(p)
    ll = [nm_to_latlong(SECTOR_CENTER, q) for q in p]
    plat = np.array([q[0] for q in ll])
    plon = np.array([q[1] for q in ll])
    wpts = sector_waypoints(p, d_units)
    min_x, max_x = min(pts[:, 0]), max(pts[:, 0])
    min_y, max_y = min(pts[:, 1]), max(pts[:, 1])
    row = np.zeros(4 + 2 * SECTOR_VMAX + 3 * N)
    row[0], row[1] = nac, len(p)
    row[2:2 + len(p)] = plat
    row[2 + SECTOR_VMAX:2 + SECTOR_VMAX + len(p)] = plon
    w0 = nm_to_latlong(SECTOR_CENTER, wpts[0])
    row[2 + 2 * SECTOR_VMAX], row[3 + 2 * SECTOR_VMAX] = w0
    base = 4 + 2 * SECTOR_VMAX
    for i in range(nac):
        for t in range(4096):
            x, y, z, w = draw(i, t)
            q = np.array([min_x + (max_x - min_x) * _u01(x, y), min_y + (max_y - min_y) * _u01(z, w)])
            q = nm_to_latlong(SECTOR_CENTER, q)
            if points_in_poly(q[0], q[1], plat, plon):
                break
        hdg = get_hdg(q, nm_to_latlong(SECTOR_CENTER, wpts[i]))
        row[base + 3 * i: base + 3 * i + 3] = q[0], q[1], hdg
    return row


# --------------------------------------------------------------------------------------
# host (parity-mode) spawn rows drawn from legacy np.random exactly as the reference envs
# consume it
# --------------------------------------------------------------------------------------
def static_spawn_from_np_random(rs, alt=350.0):
    """static_obstacle_env.py:96-124: centres (:214-226), polygons (:148-162, per obstacle
    after all centres), waypoint rejection loop (:187-212)."""
    cen = [(rs.randint(20, 150), rs.randint(0, 360)) for _ in range(STATIC_NUM_OBSTACLES)]
    row = []
    for o in range(STATIC_NUM_OBSTACLES):
        area = rs.randint(OBSTACLE_AREA_RANGE[0] * 2, OBSTACLE_AREA_RANGE[1])
        R = np.sqrt(area / np.pi)
        us = [rs.uniform(0., 1.) for _ in range(3)]
        p = sort_points_clockwise([point_on_circle(R, u) for u in us])
        while polygon_area(p) < OBSTACLE_AREA_RANGE[0]:
            us.append(rs.uniform(0., 1.))
            p.append(point_on_circle(R, us[-1]))
            p = sort_points_clockwise(p)
        assert len(us) <= STATIC_VMAX, "obstacle polygon exceeds the device vertex budget"
        row += [cen[o][0], cen[o][1], area, len(us)] + us + [0.0] * (STATIC_VMAX - len(us))
    geo = static_polygons(np.array(row + [0.0, 0.0], np.float64))
    for _ in range(1000):
        wd, wh = rs.randint(100, 170), rs.randint(0, 360)
        wlat, wlon = bsx.get_point_at_distance(52.0, 4.0, wd, wh)
        if not any(points_in_poly(wlat, wlon, pl[0], pl[1]) for pl in geo["poly"]):
            break
    return np.array(row + [wd, wh], np.float64)


def sector_spawn_from_np_random(rs, N, density_mode="normal"):
    """sector_cr_env.py:84-109: polygon (:140-158), density (:95-100), waypoints
    (:160-182), aircraft positions (:184-208)."""
    R = np.sqrt(SECTOR_POLY_AREA_RANGE[1] / np.pi)
    p = sort_points_clockwise([point_on_circle(R, rs.uniform(0., 1.)) for _ in range(3)])
    a = polygon_area(p)
    while a < SECTOR_POLY_AREA_RANGE[0]:
        p.append(point_on_circle(R, rs.uniform(0., 1.)))
        p = sort_points_clockwise(p)
        a = polygon_area(p)
    assert len(p) <= SECTOR_VMAX
    if density_mode == "normal":
        dens = rs.normal(0.005, 0.001)
    else:
        dens = rs.uniform(0.003, 0.007)
    nac = int(max(np.ceil(dens * a), 4 + 1))
    assert nac <= N, f"SectorCR episode with {nac} aircraft exceeds num_ac={N}"
    perim = 0
    for i in range(len(p)):
        perim += euclidean_distance(np.array(p[i]), np.array(p[(i + 1) % len(p)]))
    ds = [rs.uniform(0, perim) for _ in range(nac)]
    pts = np.array(p)
    min_x, max_x = min(pts[:, 0]), max(pts[:, 0])
    min_y, max_y = min(pts[:, 1]), max(pts[:, 1])
    ll = [nm_to_latlong(SECTOR_CENTER, q) for q in p]
    plat = np.array([q[0] for q in ll])
    plon = np.array([q[1] for q in ll])
    pos = []
    while len(pos) < nac:
        q = np.array([rs.uniform(min_x, max_x), rs.uniform(min_y, max_y)])
        q = nm_to_latlong(SECTOR_CENTER, q)
        if points_in_poly(q[0], q[1], plat, plon):
            pos.append(q)
    wpts = _sector_wpts_from_d(p, ds)
    row = np.zeros(4 + 2 * SECTOR_VMAX + 3 * N)
    row[0], row[1] = nac, len(p)
    row[2:2 + len(p)] = plat
    row[2 + SECTOR_VMAX:2 + SECTOR_VMAX + len(p)] = plon
    row[2 + 2 * SECTOR_VMAX: 4 + 2 * SECTOR_VMAX] = nm_to_latlong(SECTOR_CENTER, wpts[0])
    base = 4 + 2 * SECTOR_VMAX
    for i in range(nac):
        hdg = get_hdg(pos[i], nm_to_latlong(SECTOR_CENTER, wpts[i]))
        row[base + 3 * i: base + 3 * i + 3] = pos[i][0], pos[i][1], hdg
    return row


def _sector_wpts_from_d(p, ds):
    edges = []
    perim = 0
    for i in range(len(p)):
        p1 = np.array(p[i])
        p2 = np.array(p[(i + 1) % len(p)])
        le = euclidean_distance(p1, p2)
        edges.append((p1, p2, le))
        perim += le
    d_list = sorted(ds)
    wpts = []
    cur = 0
    for d in d_list:
        while d > cur + edges[0][2]:
            cur += edges[0][2]
            edges.pop(0)
        e = edges[0]
        frac = (d - cur) / e[2]
        wpts.append(e[0] + frac * (e[1] - e[0]))
    return wpts
