"""Host-side polygon helpers of StaticObstacleEnv-v0 / SectorCREnv-v0, used only to draw
host (parity-mode) spawn rows with the reference's legacy ``np.random`` consumption.

bluesky_gym/envs/common/functions.py: random_point_on_circle (:44-59), sort_points_clockwise
(:61-75), polygon_area (:77-96), nm_to_latlong (:98-114), euclidean_distance (:134-148),
get_hdg (:150-175); get_point_at_distance (:24-42) comes from config.  The areafilter POLY
test (even-odd crossings over (lat, lon) vertices) is needed here only to replay the
reference's rejection loops.  Every per-step computation (obs, reward, containment) runs
in the HIP kernel (csrc/bsg_areas.h).
"""
from __future__ import annotations

import numpy as np

from .config import get_point_at_distance

STATIC_NUM_OBSTACLES = 10
STATIC_VMAX = 16
SECTOR_VMAX = 32
SECTOR_CENTER = np.array([51.990426702297746, 4.376124857109851])


def point_on_circle(radius, u):
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
    return np.array([center[0] + (point[0] / 60),
                     center[1] + (point[1] / (60 * np.cos(np.radians(center[0]))))])


def euclidean_distance(p1, p2):
    return np.sqrt(np.sum((p2 - p1) ** 2))


def get_hdg(point1, point2):
    lat1, lon1 = np.radians(point1)
    lat2, lon2 = np.radians(point2)
    delta_lon = lon2 - lon1
    x = np.sin(delta_lon) * np.cos(lat2)
    y = np.cos(lat1) * np.sin(lat2) - np.sin(lat1) * np.cos(lat2) * np.cos(delta_lon)
    return (np.degrees(np.arctan2(x, y)) + 360) % 360


def inside(lat, lon, plat, plon):
    """Even-odd crossing test (matplotlib point_in_path), x = lat, y = lon."""
    res = False
    n = len(plat)
    for k in range(n):
        x0, y0, x1, y1 = plat[k], plon[k], plat[(k + 1) % n], plon[(k + 1) % n]
        yf0, yf1 = y0 >= lon, y1 >= lon
        if yf0 != yf1 and ((((y1 - lon) * (x0 - x1)) >= ((x1 - lat) * (y0 - y1))) == yf1):
            res = not res
    return res


def _static_ring(centre, R, us):
    p = [point_on_circle(R, u) for u in us[:3]]
    p = sort_points_clockwise(p)
    for u in us[3:]:
        p.append(point_on_circle(R, u))
        p = sort_points_clockwise(p)
    ll = [nm_to_latlong(centre, q) for q in p]
    return np.array([q[0] for q in ll]), np.array([q[1] for q in ll])


def static_spawn(rs=None):
    """static_obstacle_env.py:96-124 draws: obstacle centres (:214-226), then each polygon
    (:148-162), then the waypoint rejection loop (:187-212).  Row layout: include/bsg.h."""
    rs = np.random if rs is None else rs
    cen = [(rs.randint(20, 150), rs.randint(0, 360)) for _ in range(STATIC_NUM_OBSTACLES)]
    row, rings = [], []
    for o in range(STATIC_NUM_OBSTACLES):
        area = rs.randint(100, 1000)
        R = np.sqrt(area / np.pi)
        us = [rs.uniform(0., 1.) for _ in range(3)]
        p = sort_points_clockwise([point_on_circle(R, u) for u in us])
        while polygon_area(p) < 50:
            us.append(rs.uniform(0., 1.))
            p.append(point_on_circle(R, us[-1]))
            p = sort_points_clockwise(p)
        if len(us) > STATIC_VMAX:
            raise RuntimeError("obstacle polygon exceeds the device vertex budget (16)")
        clat, clon = get_point_at_distance(52.0, 4.0, cen[o][0], cen[o][1])
        rings.append(_static_ring((clat, clon), R, us))
        row += [cen[o][0], cen[o][1], area, len(us)] + us + [0.0] * (STATIC_VMAX - len(us))
    for _ in range(1000):
        wd, wh = rs.randint(100, 170), rs.randint(0, 360)
        wlat, wlon = get_point_at_distance(52.0, 4.0, wd, wh)
        if not any(inside(wlat, wlon, r[0], r[1]) for r in rings):
            break
    return np.array(row + [wd, wh], np.float64)


def sector_spawn(num_ac, rs=None, density_mode="normal"):
    """sector_cr_env.py:84-109 draws: polygon (:140-158), density (:95-100), waypoints
    (:160-182), aircraft positions (:184-208).  Row layout: include/bsg.h."""
    rs = np.random if rs is None else rs
    R = np.sqrt(3750 / np.pi)
    p = sort_points_clockwise([point_on_circle(R, rs.uniform(0., 1.)) for _ in range(3)])
    a = polygon_area(p)
    while a < 2400:
        p.append(point_on_circle(R, rs.uniform(0., 1.)))
        p = sort_points_clockwise(p)
        a = polygon_area(p)
    if len(p) > SECTOR_VMAX:
        raise RuntimeError("sector polygon exceeds the device vertex budget (32)")
    dens = rs.normal(0.005, 0.001) if density_mode == "normal" else rs.uniform(0.003, 0.007)
    nac = int(max(np.ceil(dens * a), 5))
    if nac > num_ac:
        raise RuntimeError(f"SectorCR episode drew {nac} aircraft > num_ac={num_ac}")
    edges, perim = [], 0
    for i in range(len(p)):
        p1, p2 = np.array(p[i]), np.array(p[(i + 1) % len(p)])
        le = euclidean_distance(p1, p2)
        edges.append((p1, p2, le))
        perim += le
    d_list = sorted(rs.uniform(0, perim) for _ in range(nac))
    wpts, cur = [], 0
    for d in d_list:
        while d > cur + edges[0][2]:
            cur += edges[0][2]
            edges.pop(0)
        e = edges[0]
        wpts.append(e[0] + ((d - cur) / e[2]) * (e[1] - e[0]))
    pts = np.array(p)
    ll = [nm_to_latlong(SECTOR_CENTER, q) for q in p]
    plat = np.array([q[0] for q in ll])
    plon = np.array([q[1] for q in ll])
    pos = []
    while len(pos) < nac:
        q = np.array([rs.uniform(min(pts[:, 0]), max(pts[:, 0])),
                      rs.uniform(min(pts[:, 1]), max(pts[:, 1]))])
        q = nm_to_latlong(SECTOR_CENTER, q)
        if inside(q[0], q[1], plat, plon):
            pos.append(q)
    row = np.zeros(4 + 2 * SECTOR_VMAX + 3 * num_ac)
    row[0], row[1] = nac, len(p)
    row[2:2 + len(p)] = plat
    row[2 + SECTOR_VMAX:2 + SECTOR_VMAX + len(p)] = plon
    row[2 + 2 * SECTOR_VMAX: 4 + 2 * SECTOR_VMAX] = nm_to_latlong(SECTOR_CENTER, wpts[0])
    base = 4 + 2 * SECTOR_VMAX
    for i in range(nac):
        w = nm_to_latlong(SECTOR_CENTER, wpts[i])
        row[base + 3 * i: base + 3 * i + 3] = pos[i][0], pos[i][1], get_hdg(pos[i], w)
    return row
