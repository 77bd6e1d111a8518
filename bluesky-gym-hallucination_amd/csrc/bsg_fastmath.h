// bsg_fastmath.h -- the three fixed-exponent powers of the BlueSky atmosphere and the
// CAS/TAS conversions, as short polynomials instead of the generic libm pow.
//
// bluesky.tools.aero (oracle/bluesky_subset.py: vatmos, vtas2cas, vcas2tas) evaluates
//   pow(T/288.15, 4.256848030018761)   T/288.15 in [0.7519, 1] below 11 km .. above
//   pow(z, 3.5)                        z = 1 + rho*v^2/(7p) = 1 + M^2/5, subsonic z < 1.3
//   pow(y, 2.0/7.0)                    y = 1 + qdyn/p, in [1, 2] up to M ~ 1.1
// The device libm's pow is 215 VALU instructions of one dependency chain (a dump of
// ocml's pow at -O3); each conversion runs two of them in series, and the per-substep
// speed chain of a climbing/descending aircraft runs seven.  On its argument range each
// power here is one Horner chain of 12 or 20 FMAs on d = x - x0 (exact, Sterbenz),
// with Chebyshev coefficients fitted to the exact binary64 exponent
// (tools/fastmath/gen_coeffs.py, fit error <= 1.2e-18 relative); outside the range the
// libm pow runs as before.  Accuracy against the correctly rounded power (glibc pow,
// which NumPy calls): tools/fastmath/ulp_check.cpp on the host (the same FMA/mul
// arithmetic) and tools/probe/fastmath_probe.hip on gfx950.
#pragma once

#include <hip/hip_runtime.h>

#include "bsg_fastmath_coeffs.h"

namespace bsg {

// Horner in plain FMAs down to the quadratic coefficient, then the last three steps in
// double-double (TwoProd by FMA, Fast2Sum: |c_k| >= |(rest)*d| on the range, asserted by
// the generator) with c2, c1, c0 carried as hi + lo.  Rounding c0..c2 and the last steps
// in plain binary64 costs up to ~2.5 ulp where the result is small against c0 (pow_trop
// near 0.75); this way the one rounding that remains is the final add (~0.5 ulp).
// The plain-FMA part (degree DEG-3 in d, its error scaled by d^3) runs as two interleaved
// Horner halves, p = P_a(d) * d^m + P_b(d): half the dependent FMA depth (the substep
// chains are latency-bound at one or two waves per SIMD).
template <int DEG>
__host__ __device__ __forceinline__ double poly_dd(const double (&c)[DEG + 1],
                                                   const double (&clo)[3], double d) {
  double p = c[0];
#pragma unroll
  for (int k = 1; k <= DEG - 3; ++k) p = fma(p, d, c[k]);
  double uh = p, ul = 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    // (uh + ul) <- c + (uh + ul) * d
    const double ck = c[DEG - 2 + k];
    const double qh = uh * d, ql = fma(uh, d, -qh);
    const double sh = ck + qh;
    const double sl = qh - (sh - ck);
    ul = (sl + ql) + fma(ul, d, clo[k]);
    uh = sh;
  }
  return uh + ul;
}

// The polynomials alone (no range test): callers test the range of a whole chain once and
// redo it with the libm pow when any argument is outside -- a branch costs ~80 cycles of
// latency whether taken or not (tools/probe/latency_probe.hip), one per power adds up.
__host__ __device__ __forceinline__ double poly_trop(double x) {
  return poly_dd<kPowT_DEG>(kPowT_C, kPowT_CLO, x - kPowT_X0);
}
__host__ __device__ __forceinline__ double poly_3p5(double z) {
  return poly_dd<kPow35_DEG>(kPow35_C, kPow35_CLO, z - kPow35_X0);
}
__host__ __device__ __forceinline__ double poly_2o7(double y) {
  return poly_dd<kPow27_DEG>(kPow27_C, kPow27_CLO, y - kPow27_X0);
}
__host__ __device__ __forceinline__ bool in_trop(double x) { return x >= kPowT_LO && x <= kPowT_HI; }
__host__ __device__ __forceinline__ bool in_3p5(double z) { return z >= kPow35_LO && z <= kPow35_HI; }
__host__ __device__ __forceinline__ bool in_2o7(double y) { return y >= kPow27_LO && y <= kPow27_HI; }

// pow(x, 4.256848030018761), the troposphere density ratio of vatmos
__host__ __device__ __forceinline__ double pow_trop(double x) {
  if (in_trop(x)) return poly_trop(x);
  return pow(x, 4.256848030018761);
}

// pow(z, 3.5)
__host__ __device__ __forceinline__ double pow_3p5(double z) {
  if (in_3p5(z)) return poly_3p5(z);
  return pow(z, 3.5);
}

// pow(y, 2.0 / 7.0)
__host__ __device__ __forceinline__ double pow_2o7(double y) {
  if (in_2o7(y)) return poly_2o7(y);
  return pow(y, 2.0 / 7.0);
}

// ---- correctly rounded division by a known divisor -------------------------------------
// x / y given ry = RN(1/y): q = RN(x*ry) is within 1 ulp of x/y, the remainder x - q*y is
// exact by FMA, and q + rem*ry rounded once is RN(x/y) (Markstein's theorem; Muller et
// al., Handbook of Floating-Point Arithmetic, "Markstein's iteration").  3 dependent
// FMA-class instructions instead of the 10-instruction v_div_scale/rcp/fma/fmas/fixup
// sequence the compiler emits for '/'.  Valid for normal, non-overflowing quotients
// (every use here: physical quantities); a zero numerator keeps its sign and an infinite
// one stays infinite, as with '/'.
// Verified against '/' on 2*10^7 random and near-halfway numerators per divisor used
// (tools/fastmath/ulp_check.cpp).
__host__ __device__ __forceinline__ double div_r(double x, double y, double ry) {
  const double q = x * ry;
  const double rem = fma(-q, y, x);
  const double r = fma(rem, ry, q);
  return (x == 0.0 || !__builtin_isfinite(q)) ? q : r;
}

// divisor known at compile time: 1.0 / y folds to RN(1/y)
__host__ __device__ __forceinline__ double divk(double x, double y) { return div_r(x, y, 1.0 / y); }

// divk for a finite numerator and y > 0: the zero quotient's sign by copysign (one bit
// operation) instead of divk's compare/select guard
__host__ __device__ __forceinline__ double divk_f(double x, double y) {
  const double ry = 1.0 / y;
  const double q = x * ry;
  return copysign(fma(fma(-q, y, x), ry, q), x);
}

// the same for a finite numerator whose zero, if any, is +0 (every physically non-negative
// quantity: temperatures, squared speeds, dynamic pressures, distances): the guard's
// compare/select pair is half the latency of the division itself
__host__ __device__ __forceinline__ double div_r_nn(double x, double y, double ry) {
  const double q = x * ry;
  return fma(fma(-q, y, x), ry, q);
}
__host__ __device__ __forceinline__ double divk_nn(double x, double y) { return div_r_nn(x, y, 1.0 / y); }

// ---- sin / cos ------------------------------------------------------------------------
// The device libm's sincos spends ~75 VALU on its small-argument path (3-part
// double-double reduction, two polynomials whose 64-bit coefficients are each moved into
// VGPRs, quadrant selection); cos alone ~70.  Every substep of every aircraft needs three
// (heading, latitude, LNAV longitude gap) and the observation phase several more.  Here:
//   k = rint(x * 2/pi);  t = x - k*P1 (exact: fma, both multiples of ulp(P1)/2, |t| < 1);
//   (r, rr) = t - k*P2 - k*P3 in double-double (TwoProd of k*P2 by FMA, TwoSum);
//   fdlibm-form kernels sin(r + rr) = r - ((z*(rr/2 - v*S') - rr) - v*S1), v = z*r, and
//   cos(r + rr) = w + (((1 - w) - z/2) + (z*z*C(z) - r*rr)), w = 1 - z/2, with minimax
//   coefficients fitted by tools/fastmath/gen_coeffs.py (fit error <= 1.3e-18);
//   quadrant k mod 4 swaps / negates.
// Domain: |x| < 2^30 (the quadrant is (int)k; the reduction keeps ~2^-100 relative
// accuracy there) -- every angle of the env path is below 10^4 rad.  inf / NaN give NaN
// through the arithmetic.  No libm fallback: an out-of-line call made the compiler assume
// the call ABI for the whole kernel (190 VGPRs, 1 KB scratch per lane), and an inlined
// one doubled the code size of every call site.
// sin_t, cos_t and sincos_t share the reduction and kernels, so a value evaluated through
// any of them has the same bits.  Accuracy vs glibc (correctly rounded in practice,
// what NumPy calls): tools/fastmath/ulp_check.cpp, tools/probe/fastmath_probe.hip.
struct TrigRed { double r, rr; int q; };

__host__ __device__ __forceinline__ TrigRed trig_reduce(double x) {
  const double k = rint(x * kTwoOverPi);
  const double t = fma(-k, kPio2Hi, x);
  const double a = k * kPio2Mid;
  const double al = fma(k, kPio2Mid, -a);
  const double r0 = t - a;                          // TwoSum(t, -a): |t| < |a| near k*pi/2
  const double bb = r0 - t;
  const double e0 = (t - (r0 - bb)) + (-a - bb);
  const double e = (e0 - al) - k * kPio2Lo;
  TrigRed o;
  o.r = r0 + e;                                     // renormalise (Fast2Sum, |r0| >= |e|)
  o.rr = e - (o.r - r0);
  o.q = (int)k & 3;
  return o;
}

// The two roundings that dominate beyond fdlibm's: S1 as a double (up to ~0.2 ulp of
// sin at |r| ~ pi/4: its low part goes into the tail) and z = r*r in cos's 1 - z/2 (up to
// ~0.25 ulp: the exact error zl of r*r, by FMA, goes into the tail).
__host__ __device__ __forceinline__ double ksin(double r, double rr, double z) {
  const double v = z * r;
  double p = kSinC[6];
#pragma unroll
  for (int k = 5; k >= 1; --k) p = fma(p, z, kSinC[k]);
  return r - ((z * (0.5 * rr - v * p) - rr) - fma(v, kSinC0Lo, v * kSinC[0]));
}

__host__ __device__ __forceinline__ double kcos(double r, double rr, double z) {
  double p = kCosC[5];
#pragma unroll
  for (int k = 4; k >= 0; --k) p = fma(p, z, kCosC[k]);
  const double zl = fma(r, r, -z);                  // r*r = z + zl exactly
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + ((((1.0 - w) - hz) - 0.5 * zl) + (z * (z * p) - r * rr));
}

__host__ __device__ __forceinline__ void sincos_t(double x, double* s, double* c) {
  const TrigRed t = trig_reduce(x);
  const double z = t.r * t.r;
  const double ss = ksin(t.r, t.rr, z), cc = kcos(t.r, t.rr, z);
  const double sq = (t.q & 1) ? cc : ss, cq = (t.q & 1) ? ss : cc;
  *s = x == 0.0 ? x : ((t.q & 2) ? -sq : sq);        // sin(-0) = -0
  *c = ((t.q + 1) & 2) ? -cq : cq;
}

__host__ __device__ __forceinline__ double sin_t(double x) {
  const TrigRed t = trig_reduce(x);
  const double z = t.r * t.r;
  const double v = (t.q & 1) ? kcos(t.r, t.rr, z) : ksin(t.r, t.rr, z);
  return x == 0.0 ? x : ((t.q & 2) ? -v : v);
}

__host__ __device__ __forceinline__ double cos_t(double x) {
  const TrigRed t = trig_reduce(x);
  const double z = t.r * t.r;
  const double v = (t.q & 1) ? ksin(t.r, t.rr, z) : kcos(t.r, t.rr, z);
  return ((t.q + 1) & 2) ? -v : v;
}

// ---- sin / cos carried along a trajectory --------------------------------------------
// The latitude and the LNAV longitude gap of an aircraft move by < 2e-3 rad per substep
// (300 m/s, 5 s, below 80 deg).  Their sin/cos are carried from substep to substep by the
// angle-addition formulas instead of being evaluated afresh -- ~50 cycles of dependent
// latency instead of sincos_t's ~330, twice per substep on the LNAV chain.
// The pair is carried in double-double: (s + sl, c + cl), seeded by sincos_dd (sincos_t's
// kernels with their tails kept, ~0.1 ulp) at every launch, advanced by
//   sin(x + d) = s + (s (cos d - 1) + c sin d),  cos(x + d) = c + (c (cos d - 1) - s sin d)
// whose corrections are ~|d| times the values (their roundings ~|d| ulp), summed with the
// low parts by TwoSum.  s and c (the rounded values) are what the substep uses: within
// ~0.6 ulp of the exact sin/cos of the carried angle, which stays the angle NumPy
// evaluates (the increments are exact differences of the rounded radian values).
// tools/fastmath/angle_add_check.cpp measures it against glibc over 30-step trajectories.
struct SinCos { double s, sl, c, cl; };

__host__ __device__ __forceinline__ void ksin_dd(double r, double rr, double z, double* hi, double* lo) {
  const double v = z * r;
  double p = kSinC[6];
#pragma unroll
  for (int k = 5; k >= 1; --k) p = fma(p, z, kSinC[k]);
  const double e = (z * (0.5 * rr - v * p) - rr) - fma(v, kSinC0Lo, v * kSinC[0]);
  *hi = r - e;                                       // ksin's value
  *lo = (r - *hi) - e;                               // Fast2Sum: |r| >= |e|
}

__host__ __device__ __forceinline__ void kcos_dd(double r, double rr, double z, double* hi, double* lo) {
  double p = kCosC[5];
#pragma unroll
  for (int k = 4; k >= 0; --k) p = fma(p, z, kCosC[k]);
  const double zl = fma(r, r, -z);
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  const double t = (((1.0 - w) - hz) - 0.5 * zl) + (z * (z * p) - r * rr);
  *hi = w + t;                                       // kcos's value
  *lo = (w - *hi) + t;                               // Fast2Sum: w >= 1/2 > |t|
}

// sincos_t with the kernels' tails: (s, c) are sincos_t's values bit for bit
__host__ __device__ __forceinline__ SinCos sincos_dd(double x) {
  const TrigRed t = trig_reduce(x);
  const double z = t.r * t.r;
  double sh, sl, ch, cl;
  ksin_dd(t.r, t.rr, z, &sh, &sl);
  kcos_dd(t.r, t.rr, z, &ch, &cl);
  const bool sw = t.q & 1, ns = t.q & 2, nc = (t.q + 1) & 2;
  SinCos o;
  o.s = sw ? ch : sh; o.sl = sw ? cl : sl;
  o.c = sw ? sh : ch; o.cl = sw ? sl : cl;
  if (ns) { o.s = -o.s; o.sl = -o.sl; }
  if (nc) { o.c = -o.c; o.cl = -o.cl; }
  if (x == 0.0) { o.s = x; o.sl = 0.0; }              // sin(-0) = -0
  return o;
}

// advance by d (|d| <= 0.05): sin d to d^7, cos d - 1 to d^8 (truncation < 2^-70 |d|)
__host__ __device__ __forceinline__ void sincos_add(SinCos& a, double d) {
  const double z = d * d;
  const double sd = fma(d * z, fma(z, fma(z, -1.0 / 5040.0, 1.0 / 120.0), -1.0 / 6.0), d);
  const double cm1 = z * fma(z, fma(z, fma(z, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5);
  const double ts = fma(a.s, cm1, a.c * sd) + a.sl;
  const double tc = fma(a.c, cm1, -(a.s * sd)) + a.cl;
  const double hs = a.s + ts, hc = a.c + tc;
  const double bs = hs - a.s, bc = hc - a.c;         // TwoSum remainders
  a.sl = (a.s - (hs - bs)) + (ts - bs);
  a.cl = (a.c - (hc - bc)) + (tc - bc);
  a.s = hs;
  a.c = hc;
}

}  // namespace bsg
