// bsg_device.h -- fp64 device math of the BlueSky subset for gfx950.
//
// Every function restates, in the same IEEE operation order, the NumPy code of
// oracle/bluesky_subset.py (itself a restatement of bluesky-simulator 1.0.3:
// bluesky/tools/aero.py, bluesky/tools/geo.py, bluesky/traffic/*.py; frozen in
// docs/BLUESKY_SUBSET_SPEC.md).  Build with -ffp-contract=off: NumPy never fuses a
// multiply-add, so neither may we.  Transcendentals come from the device libm (ocml);
// they may differ from NumPy's by an ulp, which is why fp outputs are compared with a
// tolerance while every boolean/index output is compared bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsg_fastmath.h"

namespace bsg {

// ---- constants (bluesky.tools.aero; oracle/bluesky_subset.py) -----------------------
constexpr double kPi = 3.141592653589793238462643383279502884;
constexpr double kD2R = kPi / 180.0;   // np.radians / np.deg2rad multiply by this
constexpr double kR2D = 180.0 / kPi;   // np.degrees
constexpr double Rearth = 6371000.0;
constexpr double NM = 1852.0;
constexpr double FT = 0.3048;
constexpr double KTS = 0.514444;
constexpr double FPM = 0.00508;
constexpr double G0 = 9.80665;
constexpr double RGAS = 287.05287;
constexpr double GAMMA = 1.40;
constexpr double P0 = 101325.0;
constexpr double RHO0 = 1.225;
constexpr double TSTRAT = 216.65;

// frozen A320 envelope / autopilot defaults (docs/BLUESKY_SUBSET_SPEC.md §A.3).  VMAX_CAS
// and the phase-GD envelope are fitted to the reference's SAC training logs
// (oracle/bluesky_subset.py, tests/test_ref_logs.py); VSMAX is 4000 fpm, non-binding (the
// round-2 fit was withdrawn in round 4: the held-out actors rejected it)
constexpr double TAN_BANKDEF = 0.4663076581549986;    // tan(radians(25)), frozen literal
constexpr double APVSDEF = 1500.0 * FPM;
constexpr double EPS_SPD = 0.01;
constexpr double AXMAX = 0.5;
constexpr double VMIN_CAS = 140.0 * KTS;
constexpr double VMAX_CAS = 163.0;
constexpr double MMO = 0.80;   // pinned by the reference's saved Merge states (M0.80 at 10,000 m)
constexpr double HMAX = 39800.0 * FT;
constexpr double VSMAX = 4000.0 * FPM;
constexpr double VSMIN = -4000.0 * FPM;  // unreachable: the limits see |ap.vs|
constexpr double GD_ALT_FT = 75.0;       // OpenAP phase GD: alt / ft <= 75
constexpr double VMAX_GD = 89.0;         // phase GD: CAS in [0, VMAX_GD], axmax AXMAX_GD (saved Horizontal states)
constexpr double AXMAX_GD = 2.0;
constexpr double RPZ = 5.0 * NM;
constexpr double HPZ = 1000.0 * FT;
constexpr double DTLOOKAHEAD = 300.0;

__device__ __forceinline__ uint64_t bits(double x) { return (uint64_t)__double_as_longlong(x); }

__device__ __forceinline__ double sgn(double x) { return (double)((x > 0.0) - (x < 0.0)); }

// (double)on * sgn(d) * c for c >= 0, bit for bit (the zero's sign included: -0.0 when
// d < 0), without the int -> double conversion and two multiplies.  Every use has
// on => d != 0 (on is |d| > some threshold >= 0), where sgn(d) * c = +-c.
__device__ __forceinline__ double sgnmul(bool on, double d, double c) {
  const double v = on ? c : 0.0;
  return d < 0.0 ? -v : v;
}

// np.remainder(a, 360.0) (numpy npy_divmod: fmod, then the sign fix).  |a| < 360 is every
// call but a rare one: there fmod(a, 360) = a exactly, and the result is a + 360 for
// a < 0 (npy_divmod's one rounding) or a + 0.0 otherwise (the identity, with -0 -> +0 as
// copysign(0, 360) gives).  Other |a| take the fmod path behind a branch.  (A branch-free
// exact form via trunc/FMA measured slower: its compare/select chain sits on the LNAV
// critical path, tools/probe/substep_probe.hip.)
__host__ __device__ __forceinline__ double pymod360(double a) {
  if (fabs(a) < 360.0) return a < 0.0 ? a + 360.0 : a + 0.0;
  double mod = fmod(a, 360.0);
  if (mod != 0.0) {
    if (mod < 0.0) mod += 360.0;
  } else {
    mod = 0.0;
  }
  return mod;
}

// np.maximum / np.minimum on finite inputs
__device__ __forceinline__ double npmax(double a, double b) { return (a >= b || a != a) ? a : b; }
__device__ __forceinline__ double npmin(double a, double b) { return (a <= b || a != a) ? a : b; }

__device__ __forceinline__ double degto180(double a) { return pymod360(a + 180.0) - 180.0; }

// pymod360 where the caller proves the argument's range (or NaN), without the branch
// (~150 -> 31 / 94 cycles of latency, tools/probe/latency_probe.hip):
//  - pymod360_s: a in [-360, 360) -- e.g. atan2(..) * R2D, |a| <= 180 + 1 ulp: the fast
//    path above as one select;
//  - pymod360_r: a in [-360, 720) -- e.g. a difference of two [0, 360] angles + 180:
//    a >= 360 has fmod(a, 360) = a - 360 exactly (Sterbenz: 360 <= a < 2 * 360).
__device__ __forceinline__ double pymod360_s(double a) { return a < 0.0 ? a + 360.0 : a + 0.0; }
__device__ __forceinline__ double pymod360_r(double a) {
  const double lo = a + 360.0, hi = a - 360.0;
  return a < 0.0 ? lo : (a >= 360.0 ? hi : a + 0.0);
}
// degto180(p - q) for p, q in [0, 360]: the argument p - q + 180 is in [-180, 540]
__device__ __forceinline__ double degto180_pq(double p, double q) {
  return pymod360_r((p - q) + 180.0) - 180.0;
}

// functions.py:4-22 bound_angle_positive_negative_180 (single wrap)
__device__ __forceinline__ double bound180(double a) {
  return a > 180.0 ? -(360.0 - a) : (a < -180.0 ? 360.0 + a : a);
}

// ---- aero -----------------------------------------------------------------------
struct Atmos { double p, rho, T; };

__device__ __forceinline__ Atmos vatmos(double h) {
  Atmos a;
  a.T = npmax(288.15 - 0.0065 * h, TSTRAT);
  const double x = divk_nn(a.T, 288.15);            // T >= 216.65 > 0
  const double dhstrat = npmax(0.0, h - 11000.0);
  // one branch: the troposphere at h >= 0 (T/288.15 in the polynomial's range, and
  // exp(-0.0) == 1 exactly) is every altitude the envs fly but the HMAX ceiling, whose
  // atmosphere is a constant (kAtmosHMAX_K)
  double rho = 1.225 * poly_trop(x);
  if (!(in_trop(x) && dhstrat == 0.0))
    rho = 1.225 * pow_trop(x) * (dhstrat > 0.0 ? exp(divk(-dhstrat, 6341.552161)) : 1.0);
  a.rho = rho;
  a.p = a.rho * RGAS * a.T;
  return a;
}

// vatmos of the two fixed limit altitudes the Vertical/Descent autopilot commands (selalt
// 1e6 -> allow_h = HMAX, selalt 0): the values NumPy computes (oracle/bluesky_subset.py
// vatmos; tests/test_fastmath_cpu.py checks these literals against it)
constexpr Atmos kAtmosHMAX = {0x1.27c7249336b51p+14, 0x1.37b10b426ceafp-2, 0x1.b14cccccccccdp+7};
constexpr Atmos kAtmosSL = {0x1.8bccff9dc0a57p+16, 0x1.399999999999ap+0, 0x1.2026666666666p+8};

// The same two atmospheres with what the CAS/TAS/Mach conversions of PerfModel.limits
// divide by and its RN reciprocal (host-computed: RN(7p), RN(1/RN(7p)), RN(1/p),
// RN(RN(7p)/rho), sqrt(GAMMA*RGAS*T) correctly rounded, RN(1/snd)), so that those
// divisions are Markstein's 3-link form (~17 instead of ~74 cycles each on the chain;
// tools/fastmath/ulp_check.cpp verifies each divisor against '/').
struct AtmosK { Atmos a; double p7, r_p7, r_p, k7, snd, r_snd; };
constexpr AtmosK kAtmosHMAX_K = {kAtmosHMAX, 0x1.02ce4000cfde7p+17, 0x1.fa7312a359f5cp-18,
                                 0x1.bb24b04eeeb71p-15, 0x1.a92081eb7ed42p+18,
                                 0x1.2711ca539cbf1p+8, 0x1.bc350c7fc3a97p-9};
constexpr AtmosK kAtmosSL_K = {kAtmosSL, 0x1.5a535faa0890cp+19, 0x1.7a76ee408d549p-20,
                               0x1.4b2810787baa0p-17, 0x1.1ab6ffb9d2bf5p+19,
                               0x1.544b42cc9d77cp+8, 0x1.812c3ee51ffb9p-9};

// PerfModel.limits' CAS clamp at those two atmospheres, as TAS: vcas2tas(vmin), vcas2tas(vmax)
// for the airborne envelope and for phase GD (vmin 0 -> 0), the values NumPy computes
// (tests/test_fastmath_cpu.py checks the literals against oracle/bluesky_subset.vcas2tas).
// limits() converts ap_tas to CAS, clamps, and converts back at one constant atmosphere;
// vtas2cas and vcas2tas are inverse and increasing, so the clamp is decided on ap_tas
// against these thresholds and an unclamped ap_tas is its own round trip (NumPy's round
// trip returns it within its own cancellation error, < 1e-13 relative over 60..300 m/s:
// the (1 + x)^3.5 - 1 and y^(2/7) - 1 steps).  Saves four powers, two square roots and
// two divisions on the climbing / descending aircraft's substep chain.
struct LimK { double tvmin, tvmax, tvmax_gd; };
constexpr LimK kLimHMAX = {0x1.1a6f5cb8f15bcp+7, 0x1.2959d9f9eb8a9p+8, 0x1.5933010daea59p+7};
constexpr LimK kLimSL = {0x1.2016b11c07f8ap+6, 0x1.45fffffdd454fp+7, 0x1.63ffffff427a1p+6};

// vtas2cas / vcas2tas: both powers by polynomial with one range test for the pair (a
// branch is ~80 cycles of latency even when not taken); outside, both by the libm.
__device__ __forceinline__ double tas2cas_at(double tas, const Atmos& a) {
  const double z = 1.0 + a.rho * tas * tas / (7.0 * a.p);
  double qdyn = a.p * (poly_3p5(z) - 1.0);
  double y = divk_nn(qdyn, P0) + 1.0;               // qdyn >= 0
  double yp = poly_2o7(y);
  if (!(in_3p5(z) && in_2o7(y))) {
    qdyn = a.p * (pow(z, 3.5) - 1.0);
    y = divk(qdyn, P0) + 1.0;
    yp = pow(y, 2.0 / 7.0);
  }
  const double cas = sqrt(7.0 * P0 / RHO0 * (yp - 1.0));
  return tas < 0 ? -1 * cas : cas;
}

__device__ __forceinline__ double cas2tas_at(double cas, const Atmos& a) {
  const double z = 1.0 + divk_nn(RHO0 * cas * cas, 7.0 * P0);
  double qdyn = P0 * (poly_3p5(z) - 1.0);
  double y = 1.0 + qdyn / a.p;
  double yp = poly_2o7(y);
  if (!(in_3p5(z) && in_2o7(y))) {
    qdyn = P0 * (pow(z, 3.5) - 1.0);
    y = 1.0 + qdyn / a.p;
    yp = pow(y, 2.0 / 7.0);
  }
  const double tas = sqrt(7.0 * a.p / a.rho * (yp - 1.0));
  return cas < 0 ? -1 * tas : tas;
}

__device__ __forceinline__ double sound_at(const Atmos& a) { return sqrt(GAMMA * RGAS * a.T); }

// tas2cas_at / cas2tas_at at a constant limit atmosphere (same operations, the divisions
// by the precomputed divisors; numerators rho*tas^2 and qdyn are >= 0 or +0)
__device__ __forceinline__ double tas2cas_k(double tas, const AtmosK& k) {
  const double z = 1.0 + div_r_nn(k.a.rho * tas * tas, k.p7, k.r_p7);
  double qdyn = k.a.p * (poly_3p5(z) - 1.0);
  double y = divk_nn(qdyn, P0) + 1.0;
  double yp = poly_2o7(y);
  if (!(in_3p5(z) && in_2o7(y))) {
    qdyn = k.a.p * (pow(z, 3.5) - 1.0);
    y = divk(qdyn, P0) + 1.0;
    yp = pow(y, 2.0 / 7.0);
  }
  const double cas = sqrt(7.0 * P0 / RHO0 * (yp - 1.0));
  return tas < 0 ? -1 * cas : cas;
}

__device__ __forceinline__ double cas2tas_k(double cas, const AtmosK& k) {
  const double z = 1.0 + divk_nn(RHO0 * cas * cas, 7.0 * P0);
  double qdyn = P0 * (poly_3p5(z) - 1.0);
  double y = 1.0 + div_r_nn(qdyn, k.a.p, k.r_p);
  double yp = poly_2o7(y);
  if (!(in_3p5(z) && in_2o7(y))) {
    qdyn = P0 * (pow(z, 3.5) - 1.0);
    y = 1.0 + qdyn / k.a.p;
    yp = pow(y, 2.0 / 7.0);
  }
  const double tas = sqrt(k.k7 * (yp - 1.0));
  return cas < 0 ? -1 * tas : tas;
}

// vcasormach2tas: |spd| < 2 -> Mach, else CAS
__device__ __forceinline__ double casormach2tas_at(double spd, const Atmos& a) {
  return fabs(spd) < 2.0 ? spd * sound_at(a) : cas2tas_at(spd, a);
}

// vcasormach (Traffic.cre): returns tas, cas
__device__ __forceinline__ void casormach_at(double spd, const Atmos& a, double* tas, double* cas) {
  bool ismach = (0.1 < spd) && (spd < 2.0);
  if (ismach) {
    *tas = spd * sound_at(a);
    *cas = tas2cas_at(*tas, a);
  } else {
    *tas = cas2tas_at(spd, a);
    *cas = spd;
  }
}

// ---- geo ---------------------------------------------------------------------------
// kwikqdrdist (qdr in [0,360), dist NM)
__device__ __forceinline__ void kwikqdrdist(double lata, double lona, double latb, double lonb,
                                            double* qdr, double* dist) {
  double dlat = (latb - lata) * kD2R;
  double dlon = (pymod360((lonb - lona) + 180.0) - 180.0) * kD2R;
  double cavelat = cos_t(((lata + latb) * kD2R) * 0.5);
  double dangle = sqrt(dlat * dlat + dlon * dlon * cavelat * cavelat);
  *dist = divk_nn(6371000.0 * dangle, NM);
  *qdr = pymod360_s(atan2(dlon * cavelat, dlat) * kR2D);
}

__device__ __forceinline__ double kwikdist(double lata, double lona, double latb, double lonb) {
  double dlat = (latb - lata) * kD2R;
  double dlon = (pymod360((lonb - lona) + 180.0) - 180.0) * kD2R;
  double cavelat = cos_t(((lata + latb) * kD2R) * 0.5);
  double dangle = sqrt(dlat * dlat + dlon * dlon * cavelat * cavelat);
  return divk_nn(6371000.0 * dangle, NM);
}

// kwikdist_matrix element (operation order of the matrix form, merge_env.py:195)
__device__ __forceinline__ double kwikdist_mat(double lata, double lona, double latb, double lonb) {
  double dlat = (latb - lata) * kD2R;
  double dlon = (pymod360((lonb - lona) + 180.0) - 180.0) * kD2R;
  double cavelat = cos_t(((latb + lata) * kD2R) * 0.5);
  double dangle = sqrt(dlat * dlat + (dlon * dlon) * (cavelat * cavelat));
  return divk_nn(6371000.0 * dangle, NM);
}

// kwikqdrdist_matrix element (StateBased.detect), [i][j] = from a=i to b=j
__device__ __forceinline__ void kwikqdrdist_mat(double lata, double lona, double latb, double lonb,
                                                double* qdr, double* dist) {
  double dlat = (latb - lata) * kD2R;
  double dlon = (pymod360((lonb - lona) + 180.0) - 180.0) * kD2R;
  double cavelat = cos_t(((lata + latb) * kD2R) * 0.5);
  double dangle = sqrt(dlat * dlat + (dlon * dlon) * (cavelat * cavelat));
  *dist = divk_nn(6371000.0 * dangle, NM);
  *qdr = pymod360_s(atan2(dlon * cavelat, dlat) * kR2D);
}

__device__ __forceinline__ void kwikpos(double latd1, double lond1, double qdr, double dist,
                                        double* lat2, double* lon2) {
  double dx = dist * sin_t(qdr * kD2R);
  double dy = dist * cos_t(qdr * kD2R);
  double dlat = divk(dy, 60.0);
  double dlon = dx / npmax(0.01, 60.0 * cos_t(latd1 * kD2R));
  *lat2 = latd1 + dlat;
  *lon2 = pymod360((lond1 + dlon) + 180.0) - 180.0;
}

__device__ __forceinline__ double rwgs84(double latd) {
  double lat = latd * kD2R;
  const double a = 6378137.0;
  const double b = 6356752.314245;
  double coslat, sinlat;
  sincos_t(lat, &sinlat, &coslat);
  double an = a * a * coslat;
  double bn = b * b * sinlat;
  double ad = a * coslat;
  double bd = b * sinlat;
  return sqrt((an * an + bn * bn) / (ad * ad + bd * bd));
}

// geo.qdrdist (WGS84): qdr in (-180,180], dist NM
__device__ __forceinline__ void qdrdist(double latd1, double lond1, double latd2, double lond2,
                                        double* qdr, double* distnm) {
  bool sw = (latd1 * latd2 >= 0.0);
  double r;
  if (sw) {
    r = rwgs84(0.5 * (latd1 + latd2));
  } else {
    const double a = 6378137.0;
    double r1 = rwgs84(latd1);
    double r2 = rwgs84(latd2);
    r = 0.5 * (fabs(latd1) * (r1 + a) + fabs(latd2) * (r2 + a)) /
        npmax(0.000001, fabs(latd1) + fabs(latd2));
  }
  double lat1 = latd1 * kD2R, lon1 = lond1 * kD2R;
  double lat2 = latd2 * kD2R, lon2 = lond2 * kD2R;
  double coslat1 = cos_t(lat1), coslat2 = cos_t(lat2);
  double sinlat1 = sin_t(lat1), sinlat2 = sin_t(lat2);
  double cosdlon = cos_t(lon2 - lon1);
  double d = r * acos(coslat1 * coslat2 * cosdlon + sinlat1 * sinlat2);
  *qdr = atan2(sin_t(lon2 - lon1) * coslat2, coslat1 * sinlat2 - sinlat1 * coslat2 * cosdlon) * kR2D;
  *distnm = d / NM;
}

// geo.qdrdist for the LNAV hot loop, same arithmetic as qdrdist() with the trig terms
// that do not change between calls passed in: (coslat1, sinlat1) of the aircraft
// (carried over from update_pos, which evaluates cos/sin of the same latitude) and
// (coslat2, sinlat2) of the active waypoint (cached per waypoint).  sincos() is
// bit-identical to separate sin()/cos() on gfx950/ROCm 7.2 (tools/probe/sincos_probe.hip).
__device__ __forceinline__ bool b_times_dphi_far(double latd1, double latd2, double far_m) {
  const double bmin = 6356752.314245;                       // WGS84 minor semi-axis
  return bmin * (fabs(latd2 - latd1) * kD2R) * 0.999999 > far_m;
}

// First half of geo.qdrdist for the LNAV loop: the bearing (as qdrdist) and the acos
// argument x of its distance (the argument the full path passes to acos), given the
// longitude gap's sin/cos (sdl, cdl of lond2 * D2R - lond1 * D2R).
__device__ __forceinline__ void qdr_x_t(double coslat1, double sinlat1, double coslat2, double sinlat2,
                                        double sdl, double cdl, double* qdr, double* x) {
#if defined(BSG_EXP_FASTATAN) && BSG_EXP_FASTATAN
  // timing experiment only (wrong results): the bearing's atan2 replaced by a division
  const double yy = sdl * coslat2, xx = coslat1 * sinlat2 - sinlat1 * coslat2 * cdl;
  *qdr = (yy / (fabs(xx) + fabs(yy))) * 90.0 + (xx < 0.0 ? 180.0 : 0.0);
#else
  *qdr = atan2(sdl * coslat2, coslat1 * sinlat2 - sinlat1 * coslat2 * cdl) * kR2D;
#endif
  *x = coslat1 * coslat2 * cdl + sinlat1 * sinlat2;
}

// true when the distance qdrdist would compute from x is provably beyond far_m:
//  - the meridian gap alone: great-circle >= r*|dphi|, r >= b (1e-6 relative margin);
//  - x itself: with t = far_m/b, x < 1 - t^2/2 <= cos(t) gives acos(x) > t, so
//    d >= b*t = far_m (the 1e-12 margin covers acos's ulp error; the caller's thresholds
//    sit >= 1 m inside far_m).
__device__ __forceinline__ bool far_of(double latd1, double latd2, double x, double far_m) {
  const double t = far_m * (1.0 / 6356752.314245);
  return b_times_dphi_far(latd1, latd2, far_m) || x < (1.0 - 0.5 * t * t) - 1e-12;
}

// Second half: the distance (NM) exactly as geo.qdrdist computes it from the same x.
__device__ __forceinline__ double qdrdist_exact_nm(double latd1, double latd2, double x) {
  bool sw = (latd1 * latd2 >= 0.0);
  double r;
  if (sw) {
    r = rwgs84(0.5 * (latd1 + latd2));
  } else {
    const double a = 6378137.0;
    double r1 = rwgs84(latd1);
    double r2 = rwgs84(latd2);
    r = 0.5 * (fabs(latd1) * (r1 + a) + fabs(latd2) * (r2 + a)) /
        npmax(0.000001, fabs(latd1) + fabs(latd2));
  }
  double d = r * acos(x);
  return divk_nn(d, NM);                      // d >= 0
}

// Squared bounds [lo2, hi2] (m^2) on the distance the exact path would yield, (d/NM)*NM
// with d = rwgs84(mid-latitude) * acos(x), from x and the waypoint's radius rw -- no
// sqrt, acos, sincos or division (each a 100-300 cycle link of the LNAV chain):
//   r:    |d rwgs84 / d phi| <= a - b < 21,500 m/rad, so r(mid) is within
//         21,500 * |phi_mid - phi_wp| of r(wp) = rw (host value, +-1e-6 m for the device's
//         rounding of rwgs84 and of rw);
//   acos: acos(1 - u) = 2 asin(sqrt(u/2)) in [sqrt(2u), sqrt(2u) (1 + 0.085 u)] for
//         u <= 0.02 (asin y <= y (1 + 0.1675 y^2) at y <= 0.1), u = 1 - x exact (Sterbenz);
//   the 3e-12 relative slack covers acos's ulp error, the /NM*NM round trip and the
//   rounding of these products (each ~1e-16).
// false (decide exactly): different hemispheres (the other rwgs84 branch) or u outside
// (0, 0.02] -- x >= 1 (acos 0 or NaN) or beyond ~90 km, where LNAV never asks.
// (Straight-line: the bounds are computed whatever the validity, which is returned.)
__device__ __forceinline__ bool qdrdist_bounds2(double latd1, double latd2, double x, double rw,
                                                double* lo2, double* hi2) {
  const double u = 1.0 - x;
  const bool ok = (latd1 * latd2 >= 0.0) && (u > 0.0 && u <= 0.02);
  const double dr = 21500.0 * (0.5 * fabs(latd1 - latd2) * kD2R) + 1e-6;
  const double rlo = rw - dr, rhi = rw + dr;
  const double q = 2.0 * u;
  const double f = 1.0 + 0.085 * u;
  *lo2 = (rlo * rlo) * q * (1.0 - 3e-12);
  *hi2 = (rhi * rhi) * q * (f * f) * (1.0 + 3e-12);
  return ok;
}

// functions.py:24-42 get_point_at_distance (R = 6371 km)
__device__ __forceinline__ void get_point_at_distance(double lat1d, double lon1d, double d,
                                                      double bearing, double* lat2d, double* lon2d) {
  const double R = 6371.0;
  double lat1 = lat1d * kD2R;
  double lon1 = lon1d * kD2R;
  double a = bearing * kD2R;
  double lat2 = asin(sin_t(lat1) * cos_t(d / R) + cos_t(lat1) * sin_t(d / R) * cos_t(a));
  double lon2 = lon1 + atan2(sin_t(a) * sin_t(d / R) * cos_t(lat1), cos_t(d / R) - sin_t(lat1) * sin_t(lat2));
  *lat2d = lat2 * kR2D;
  *lon2d = lon2 * kR2D;
}

// ---- Philox4x32-10 (oracle/philox.py) ---------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

__device__ __forceinline__ double u01_53(uint32_t lo, uint32_t hi) {
  uint64_t x = ((uint64_t)hi << 32) | lo;
  return (double)(x >> 11) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ int64_t randint_u32(uint32_t x, int64_t lo, int64_t hi) {
  return lo + (((int64_t)x * (hi - lo)) >> 32);
}

constexpr uint32_t TAG_MERGE = 0x4D455247u;
constexpr uint32_t TAG_VERT = 0x56455254u;
constexpr uint32_t TAG_DESC = 0x44455343u;
constexpr uint32_t TAG_HORZ = 0x484F525Au;

}  // namespace bsg
