// Host accuracy check of bsg_fastmath.h sincos_dd / sincos_add (container-only dev tool, no GPU): the
// sin/cos of an angle carried through K increments by the angle-addition formulas against
// glibc's sin/cos of the same angle (what NumPy computes at every substep), after 1..K
// steps.  Angles and increments as the substep loop sees them: latitudes in [-80, 80] deg
// and LNAV longitude gaps in [-3, 3] deg, increments up to 2e-3 rad (300 m/s x 5 s at
// 80 deg latitude), K = 30 (Descent/Vertical substeps per RL step).
//   hipcc -O2 -x hip --offload-arch=gfx950 tools/fastmath/angle_add_check.cpp -o /tmp/aac && /tmp/aac
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../bluesky-gym-hallucination_amd/csrc/bsg_fastmath.h"

static int64_t ord(double v) {
  int64_t i;
  std::memcpy(&i, &v, 8);
  return i < 0 ? INT64_MIN - i : i;
}

int main() {
  std::mt19937_64 rng(5);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  const int K = 30, T = 200000;
  long hist[2][4] = {{0}};                  // [sin|cos][0, 1, 2, >2 ulp] over all steps
  long worst[2] = {0, 0};
  double worst_abs = 0.0;                   // |error| in units of 2^-53 (absolute, for |v| ~ 1)
  for (int t = 0; t < T; ++t) {
    const bool gap = t & 1;
    double x = gap ? 3.0 * U(rng) * (M_PI / 180) : 80.0 * U(rng) * (M_PI / 180);
    const double step = 2e-3 * U(rng);
    bsg::SinCos sc = bsg::sincos_dd(x);
    double s0, c0;
    bsg::sincos_t(x, &s0, &c0);
    if (s0 != sc.s || c0 != sc.c) { std::printf("sincos_dd != sincos_t at %a\n", x); return 1; }
    for (int k = 0; k < K; ++k) {
      const double xn = x + step * (1.0 + 0.1 * U(rng));
      bsg::sincos_add(sc, xn - x);
      x = xn;
      const double s = sc.s, c = sc.c;
      const double rs = std::sin(x), rc = std::cos(x);
      const long ds = std::labs((long)(ord(s) - ord(rs))), dc = std::labs((long)(ord(c) - ord(rc)));
      hist[0][ds > 2 ? 3 : ds]++;
      hist[1][dc > 2 ? 3 : dc]++;
      worst[0] = ds > worst[0] ? ds : worst[0];
      worst[1] = dc > worst[1] ? dc : worst[1];
      const double ea = std::fmax(std::fabs(s - rs), std::fabs(c - rc)) * 9007199254740992.0;
      worst_abs = ea > worst_abs ? ea : worst_abs;
    }
  }
  const char* nm[2] = {"sin", "cos"};
  for (int f = 0; f < 2; ++f) {
    const double n = (double)T * K;
    std::printf("%s: 0 ulp %.4f  1 ulp %.4f  2 ulp %.4f  >2 ulp %.6f  (max %ld ulp)\n", nm[f],
                hist[f][0] / n, hist[f][1] / n, hist[f][2] / n, hist[f][3] / n, worst[f]);
  }
  std::printf("max absolute error %.2f x 2^-53 over %d x %d steps\n", worst_abs, T, K);
  return 0;
}
