// bsg_areas.h -- polygons of StaticObstacleEnv-v0 / SectorCREnv-v0 on the device.
//
// Restates bluesky_gym/envs/common/functions.py (random_point_on_circle :44-59,
// sort_points_clockwise :61-75, polygon_area :77-96, nm_to_latlong :98-114, get_hdg
// :150-175) and the areafilter POLY containment test (matplotlib Path.contains_points:
// even-odd crossings, x = lat, y = lon); oracle: oracle/areas.py.
//
// Per-env geometry lives in bsg_buffers.env_geom (f64, geom_width doubles per env):
//   StaticObstacle: [0] wpt lat, [1] wpt lon, then per obstacle o at 2 + o*SO_W:
//                   clat, clon, R (NM), nvert, half-height (deg lat), half-width (deg lon),
//                   lat[SO_VMAX], lon[SO_VMAX]
//   SectorCR      : [0] num_ac, [1] nvert, [2] wpt lat, [3] wpt lon, lat[SC_VMAX], lon[SC_VMAX]
#pragma once

#include "bsg_device.h"

namespace bsg {

constexpr int SO_NOBST = 10;               // static_obstacle_env.py:37 NUM_OBSTACLES
constexpr int SO_VMAX = 16;
constexpr int SO_HDR = 6;
constexpr int SO_W = SO_HDR + 2 * SO_VMAX;
constexpr int SO_GEOM = 2 + SO_NOBST * SO_W;
constexpr int SO_SPAWN_W = SO_NOBST * (4 + SO_VMAX) + 2;
constexpr int SC_VMAX = 32;
constexpr int SC_GEOM = 4 + 2 * SC_VMAX;
constexpr int PW_NWPT = 5;                 // plan_waypoint_env.py:15 NUM_WAYPOINTS
constexpr int PW_GEOM = 2 * PW_NWPT;        // waypoint lat[5], lon[5]
constexpr uint32_t TAG_STAT = 0x53544154u;  // 'STAT'
constexpr uint32_t TAG_PLAN = 0x504C414Eu;  // 'PLAN'
constexpr uint32_t TAG_SECT = 0x53454354u;  // 'SECT'
constexpr double TWO_PI = 2.0 * 3.141592653589793;
constexpr double SC_CLAT = 51.990426702297746;   // sector_cr_env.py:16 CENTER
constexpr double SC_CLON = 4.376124857109851;

// one edge (x0,y0)->(x1,y1) of the even-odd crossing test for point (tx, ty)
__device__ __forceinline__ bool edge_crosses(double x0, double y0, double x1, double y1,
                                             double tx, double ty) {
  const bool yflag0 = y0 >= ty, yflag1 = y1 >= ty;
  return (yflag0 != yflag1) && ((((y1 - ty) * (x0 - x1)) >= ((x1 - tx) * (y0 - y1))) == yflag1);
}

// areafilter checkInside for a ring of n (lat, lon) vertices
__device__ __forceinline__ bool point_in_ring(const double* plat, const double* plon, int n,
                                              double lat, double lon) {
  bool inside = false;
  double x0 = plat[n - 1], y0 = plon[n - 1];
  for (int k = 0; k < n; ++k) {
    const double x1 = plat[k], y1 = plon[k];
    inside ^= edge_crosses(x0, y0, x1, y1, lat, lon);
    x0 = x1;
    y0 = y1;
  }
  return inside;
}

__device__ __forceinline__ double ring_area(const double* px, const double* py, int n) {
  double area = 0.0;
  for (int i = 0; i < n; ++i) {
    const int i2 = (i + 1) % n;
    area = area + (px[i] * py[i2] - py[i] * px[i2]);
  }
  return fabs(area) / 2.0;
}

// insert point (x, y) into the angle-sorted ring px/py[0..n) (np.argsort of arctan2 over
// the appended list: ties keep insertion order)
__device__ __forceinline__ void ring_insert(double* px, double* py, int n, double x, double y) {
  const double a = atan2(y, x);
  int pos = n;
  while (pos > 0 && atan2(py[pos - 1], px[pos - 1]) > a) {
    px[pos] = px[pos - 1];
    py[pos] = py[pos - 1];
    --pos;
  }
  px[pos] = x;
  py[pos] = y;
}

// functions.py polygon construction on a circle of radius R (NM) from the uniform draws
// ufn(k): the first 3 points, then one more while the area is below min_area (at most
// nmax points).  fixed_n >= 3 uses exactly that many points (host-drawn parameters).
template <class UFN>
__device__ __forceinline__ int build_ring(double* px, double* py, double R, UFN ufn, int nmax,
                                          double min_area, int fixed_n, double* area_out) {
  int n = 0;
  double area = 0.0;
  for (int k = 0; k < nmax; ++k) {
    if (fixed_n >= 3 ? k >= fixed_n : (k >= 3 && area >= min_area)) break;
    const double alpha = TWO_PI * ufn(k);
    ring_insert(px, py, n, R * cos_t(alpha), R * sin_t(alpha));
    ++n;
    if (n >= 3) area = ring_area(px, py, n);
  }
  *area_out = area;
  return n;
}

// functions.py:150-175 get_hdg
__device__ __forceinline__ double get_hdg(double lat1d, double lon1d, double lat2d, double lon2d) {
  const double lat1 = lat1d * kD2R, lon1 = lon1d * kD2R, lat2 = lat2d * kD2R, lon2 = lon2d * kD2R;
  const double dlon = lon2 - lon1;
  const double x = sin_t(dlon) * cos_t(lat2);
  const double y = cos_t(lat1) * sin_t(lat2) - sin_t(lat1) * cos_t(lat2) * cos_t(dlon);
  return pymod360(atan2(x, y) * kR2D + 360.0);
}

// ---- StaticObstacleEnv-v0 ----------------------------------------------------------------
// number of obstacles containing (lat, lon) (static_obstacle_env.py:326-337); the box test
// is exact: every vertex lies within R/60 deg lat and R/(60 cos clat) deg lon of the centre
__device__ __forceinline__ int static_inside_count(const double* geo, double lat, double lon) {
  int n = 0;
  for (int o = 0; o < SO_NOBST; ++o) {
    const double* g = geo + 2 + o * SO_W;
    if (fabs(lat - g[0]) > g[4] || fabs(lon - g[1]) > g[5]) continue;
    n += point_in_ring(g + SO_HDR, g + SO_HDR + SO_VMAX, (int)g[3], lat, lon) ? 1 : 0;
  }
  return n;
}

// static_obstacle_env.py:96-124 + _generate_obstacles :164-185 + _generate_polygon :148-162
// + _generate_waypoint :187-212 (spawn row: per obstacle dis, hdg, area, nvert, u[16]; then
// waypoint dis, hdg -- or Philox draws keyed (env, episode, draw, 'STAT')).  Writes the
// geometry; returns the waypoint.
__device__ __forceinline__ void static_build(double* geo, const double* row, uint32_t env,
                                             uint32_t episode, uint64_t seed) {
  for (int o = 0; o < SO_NOBST; ++o) {
    double dis, hdg, area_i;
    int fixed_n = 0;
    if (row) {
      const double* q = row + o * (4 + SO_VMAX);
      dis = q[0]; hdg = q[1]; area_i = q[2]; fixed_n = (int)q[3];
    } else {
      U4 r = philox4x32_10(env, episode, (uint32_t)o, TAG_STAT, seed);
      dis = (double)randint_u32(r.x, 20, 150);
      hdg = (double)randint_u32(r.y, 0, 360);
      area_i = (double)randint_u32(r.z, 100, 1000);
    }
    double clat, clon;
    get_point_at_distance(52.0, 4.0, dis, hdg, &clat, &clon);
    const double R = sqrt(area_i / 3.141592653589793);
    double* g = geo + 2 + o * SO_W;
    double* px = g + SO_HDR;
    double* py = g + SO_HDR + SO_VMAX;
    double area;
    auto ufn = [&](int k) -> double {
      if (row) return row[o * (4 + SO_VMAX) + 4 + k];
      U4 r = philox4x32_10(env, episode, (uint32_t)(16 + o * SO_VMAX + k), TAG_STAT, seed);
      return u01_53(r.x, r.y);
    };
    const int n = build_ring(px, py, R, ufn, SO_VMAX, 50.0, fixed_n, &area);
    const double ccos = 60.0 * cos_t(clat * kD2R);
    for (int k = 0; k < n; ++k) {              // nm_to_latlong(centre, point)
      px[k] = clat + (px[k] / 60.0);
      py[k] = clon + (py[k] / ccos);
    }
    g[0] = clat; g[1] = clon; g[2] = R; g[3] = (double)n;
    g[4] = (R / 60.0) * (1.0 + 1e-9) + 1e-9;
    g[5] = (R / ccos) * (1.0 + 1e-9) + 1e-9;
  }
  double wd = 0.0, wh = 0.0;
  if (row) {
    wd = row[SO_NOBST * (4 + SO_VMAX)];
    wh = row[SO_NOBST * (4 + SO_VMAX) + 1];
  } else {
    for (int t = 0; t < 1000; ++t) {
      U4 r = philox4x32_10(env, episode, (uint32_t)(1000 + t), TAG_STAT, seed);
      wd = (double)randint_u32(r.x, 100, 170);
      wh = (double)randint_u32(r.y, 0, 360);
      double la, lo;
      get_point_at_distance(52.0, 4.0, wd, wh, &la, &lo);
      if (static_inside_count(geo, la, lo) == 0) break;
    }
  }
  get_point_at_distance(52.0, 4.0, wd, wh, &geo[0], &geo[1]);
}

// ---- SectorCREnv-v0 ------------------------------------------------------------------------
struct SectorPlan {                      // per env (LDS), device-drawn resets only
  double px[SC_VMAX], py[SC_VMAX];       // sector ring in NM about CENTER (angle-sorted)
  double d[64];                          // waypoint perimeter distance by aircraft rank
  double draw[64];                       // waypoint perimeter distance by aircraft draw
  double perim, minx, maxx, miny, maxy;
  int nv, nac;
  int over;                              // the drawn count exceeded the capacity N
};

__device__ __forceinline__ void nm_to_latlong_sector(double x, double y, double* lat, double* lon) {
  *lat = SC_CLAT + (x / 60.0);
  *lon = SC_CLON + (y / (60.0 * cos_t(SC_CLAT * kD2R)));
}

// lane 0 of a resetting env: polygon (sector_cr_env.py:140-158), aircraft count (:95-100),
// perimeter and bounding box; writes the polygon and count into the env geometry
__device__ __forceinline__ void sector_plan_polygon(SectorPlan& P, double* geo, uint32_t env,
                                                    uint32_t ep, uint64_t seed, int N, int mode) {
  auto ufn = [&](int k) -> double {
    U4 r = philox4x32_10(env, ep, (uint32_t)k, TAG_SECT, seed);
    return u01_53(r.x, r.y);
  };
  double area;
  const int nv = build_ring(P.px, P.py, sqrt(3750.0 / 3.141592653589793), ufn, SC_VMAX, 2400.0,
                            0, &area);
  U4 r = philox4x32_10(env, ep, 64u, TAG_SECT, seed);
  double dens;
  if (mode == 0) {                       // np.random.normal(0.005, 0.001) via Box-Muller
    const double u1 = 1.0 - u01_53(r.x, r.y);
    const double u2 = u01_53(r.z, r.w);
    dens = 0.005 + 0.001 * (sqrt(-2.0 * log(u1)) * cos_t(TWO_PI * u2));
  } else {                               // np.random.uniform(0.003, 0.007)
    dens = 0.003 + (0.007 - 0.003) * u01_53(r.x, r.y);
  }
  int nac = (int)npmax(ceil(dens * area), 5.0);
  P.over = nac > N;                      // flagged (BSG_FLAG_SPAWN_OVERFLOW), not silent
  if (nac > N) nac = N;
  double perim = 0.0, minx = P.px[0], maxx = P.px[0], miny = P.py[0], maxy = P.py[0];
  for (int i = 0; i < nv; ++i) {
    const int i2 = (i + 1) % nv;
    const double dx = P.px[i2] - P.px[i], dy = P.py[i2] - P.py[i];
    perim = perim + sqrt(dx * dx + dy * dy);
    minx = npmin(minx, P.px[i]); maxx = npmax(maxx, P.px[i]);
    miny = npmin(miny, P.py[i]); maxy = npmax(maxy, P.py[i]);
  }
  P.nv = nv; P.nac = nac; P.perim = perim;
  P.minx = minx; P.maxx = maxx; P.miny = miny; P.maxy = maxy;
  geo[0] = (double)nac;
  geo[1] = (double)nv;
  for (int k = 0; k < nv; ++k) nm_to_latlong_sector(P.px[k], P.py[k], &geo[4 + k], &geo[4 + SC_VMAX + k]);
}

// waypoint of the aircraft whose perimeter distance is d (sector_cr_env.py:173-182)
__device__ __forceinline__ void sector_waypoint(const SectorPlan& P, double d, double* x, double* y) {
  double cur = 0.0;
  int e = 0;
  for (;;) {
    const int e2 = (e + 1) % P.nv;
    const double dx = P.px[e2] - P.px[e], dy = P.py[e2] - P.py[e];
    const double len = sqrt(dx * dx + dy * dy);
    if (d > cur + len && e < P.nv - 1) { cur += len; ++e; continue; }
    const double frac = (d - cur) / len;
    *x = P.px[e] + frac * (P.px[e2] - P.px[e]);
    *y = P.py[e] + frac * (P.py[e2] - P.py[e]);
    return;
  }
}

// initial position of aircraft j: uniform in the bounding box until inside the sector
// (sector_cr_env.py:193-199; Philox stream (env, ep, 0x10000 + 4096 j + t))
__device__ __forceinline__ void sector_position(const SectorPlan& P, const double* geo, uint32_t env,
                                                uint32_t ep, uint64_t seed, int j, double* lat,
                                                double* lon) {
  const int nv = (int)geo[1];
  for (int t = 0; t < 4096; ++t) {
    U4 r = philox4x32_10(env, ep, (uint32_t)(0x10000 + j * 4096 + t), TAG_SECT, seed);
    const double x = P.minx + (P.maxx - P.minx) * u01_53(r.x, r.y);
    const double y = P.miny + (P.maxy - P.miny) * u01_53(r.z, r.w);
    nm_to_latlong_sector(x, y, lat, lon);
    if (point_in_ring(geo + 4, geo + 4 + SC_VMAX, nv, *lat, *lon)) return;
  }
}

}  // namespace bsg
