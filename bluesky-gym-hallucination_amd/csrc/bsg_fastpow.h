// bsg_fastpow.h -- the three fixed-exponent powers of the BlueSky atmosphere and the
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
// (tools/fastpow/gen_coeffs.py, fit error <= 1.2e-18 relative); outside the range the
// libm pow runs as before.  Accuracy against the correctly rounded power (glibc pow,
// which NumPy calls): tools/fastpow/ulp_check.cpp on the host (the same FMA/mul
// arithmetic) and tools/probe/fastpow_probe.hip on gfx950.
#pragma once

#include <hip/hip_runtime.h>

#include "bsg_fastpow_coeffs.h"

namespace bsg {

// Horner in plain FMAs down to the quadratic coefficient, then the last three steps in
// double-double (TwoProd by FMA, Fast2Sum: |c_k| >= |(rest)*d| on the range, asserted by
// the generator) with c2, c1, c0 carried as hi + lo.  Rounding c0..c2 and the last steps
// in plain binary64 costs up to ~2.5 ulp where the result is small against c0 (pow_trop
// near 0.75); this way the one rounding that remains is the final add (~0.5 ulp).
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

// pow(x, 4.256848030018761), the troposphere density ratio of vatmos
__host__ __device__ __forceinline__ double pow_trop(double x) {
  if (x >= kPowT_LO && x <= kPowT_HI) return poly_dd<kPowT_DEG>(kPowT_C, kPowT_CLO, x - kPowT_X0);
  return pow(x, 4.256848030018761);
}

// pow(z, 3.5)
__host__ __device__ __forceinline__ double pow_3p5(double z) {
  if (z >= kPow35_LO && z <= kPow35_HI) return poly_dd<kPow35_DEG>(kPow35_C, kPow35_CLO, z - kPow35_X0);
  return pow(z, 3.5);
}

// pow(y, 2.0 / 7.0)
__host__ __device__ __forceinline__ double pow_2o7(double y) {
  if (y >= kPow27_LO && y <= kPow27_HI) return poly_dd<kPow27_DEG>(kPow27_C, kPow27_CLO, y - kPow27_X0);
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
// (tools/fastpow/ulp_check.cpp).
__host__ __device__ __forceinline__ double div_r(double x, double y, double ry) {
  const double q = x * ry;
  const double rem = fma(-q, y, x);
  const double r = fma(rem, ry, q);
  return (x == 0.0 || !__builtin_isfinite(q)) ? q : r;
}

// divisor known at compile time: 1.0 / y folds to RN(1/y)
__host__ __device__ __forceinline__ double divk(double x, double y) { return div_r(x, y, 1.0 / y); }

}  // namespace bsg
