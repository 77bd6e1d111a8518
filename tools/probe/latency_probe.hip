// Probe on gfx950: dependent-chain latency (shader cycles per link) of the fp64 operations
// the step kernel's per-aircraft chain is made of, one wave on an otherwise idle chip
// (the regime of a C4 shard: 512 envs = 256 waves on 1,024 SIMDs).  Each kernel runs
// ITER links x = op(x) in one lane-parallel wave and stamps s_memtime around the loop.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/probe/latency_probe.hip -o tools/probe/latency_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../../bluesky-gym-hallucination_amd/csrc/bsg_device.h"

constexpr int ITER = 2048;

#define PROBE(NAME, ...)                                                              \
  __global__ void NAME(const double* in, double* out, long long* cyc) {                \
    double x = in[threadIdx.x], a = in[64], b = in[65];                                \
    (void)a; (void)b;                                                                  \
    const long long t0 = __builtin_amdgcn_s_memtime();                                 \
    for (int i = 0; i < ITER; ++i) { __VA_ARGS__; }                                         \
    const long long t1 = __builtin_amdgcn_s_memtime();                                 \
    out[threadIdx.x] = x;                                                              \
    if (threadIdx.x == 0) cyc[0] = t1 - t0;                                            \
  }

PROBE(k_empty, x = x + 0.0)
PROBE(k_fma, x = fma(x, a, b))
PROBE(k_mul, x = x * a)
PROBE(k_add, x = x + a)
PROBE(k_div, x = a / x)
PROBE(k_divk, x = bsg::divk(x, 6371000.0) + a)
PROBE(k_sqrt, x = sqrt(x + a))
PROBE(k_rint, x = rint(x * a) + b)
PROBE(k_ocml_sincos, { double s, c; sincos(x, &s, &c); x = s + c * a; })
PROBE(k_sincos_t, { double s, c; bsg::sincos_t(x, &s, &c); x = s + c * a; })
PROBE(k_ocml_cos, x = cos(x) + a)
PROBE(k_cos_t, x = bsg::cos_t(x) + a)
PROBE(k_ocml_atan2, x = atan2(x, a) + b)
PROBE(k_pow_ocml, x = pow(x * a + 1.0, 3.5) * b)
PROBE(k_pow_3p5, x = bsg::pow_3p5(x * a + 1.0) * b)
PROBE(k_cvt_f32, x = (double)(float)x + a)
PROBE(k_select, x = (x > a) ? x * b : x + b)
PROBE(k_branch, if (x > a) { x = x * b; } else { x = x + b; })
PROBE(k_branch_skip, if (x < -1e30) { double sv, cv; sincos(x, &sv, &cv); x = sv * cv; } x = fma(x, a, b))
PROBE(k_branch_skip2, if (x < -1e30) { double sv, cv; sincos(x, &sv, &cv); x = sv * cv; } x = fma(x, a, b);
                      if (x < -1e31) { double sv, cv; sincos(x, &sv, &cv); x = sv + cv; } x = fma(x, a, b))
PROBE(k_pymod360, x = bsg::pymod360(x * 360.0 + a) * (1.0 / 360.0))
PROBE(k_branch_expect, if (__builtin_expect(x < -1e30, 0)) { double sv, cv; sincos(x, &sv, &cv); x = sv * cv; } x = fma(x, a, b))
PROBE(k_branch_ballot, if (__builtin_amdgcn_ballot_w64(x < -1e30) != 0) { double sv, cv; sincos(x, &sv, &cv); x = sv * cv; } x = fma(x, a, b))
PROBE(k_branch_any, if (__any(x < -1e30)) { if (x < -1e30) { double sv, cv; sincos(x, &sv, &cv); x = sv * cv; } } x = fma(x, a, b))
PROBE(k_cmp_sel2, x = (x > a) ? ((x > b) ? x * a : x + a) : x + b)
PROBE(k_pymod360_s, x = bsg::pymod360_s(x * 360.0 - a) * (1.0 / 360.0))
PROBE(k_pymod360_r, x = bsg::pymod360_r(x * 360.0 + a) * (1.0 / 360.0))
// a wave-uniform flag computed before the loop (an SGPR): the branch needs no VALU result
__global__ void k_branch_uniform(const double* in, double* out, long long* cyc) {
  double x = in[threadIdx.x], a = in[64], b = in[65];
  const bool u = __builtin_amdgcn_readfirstlane(in[66] > 0.5 ? 1 : 0) != 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITER; ++i) {
    if (u) { double sv, cv; sincos(x, &sv, &cv); x = sv * cv; }
    x = fma(x, a, b);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  std::vector<double> h(67, 0.3);
  h[64] = 0.999;
  h[65] = 1e-3;
  h[66] = 0.0;
  double *din, *dout;
  long long* dc;
  if (hipMalloc(&din, 67 * 8) != hipSuccess || hipMalloc(&dout, 64 * 8) != hipSuccess ||
      hipMalloc(&dc, 8) != hipSuccess)
    return 1;
  (void)hipMemcpy(din, h.data(), 67 * 8, hipMemcpyHostToDevice);
  struct K { const char* n; void (*f)(const double*, double*, long long*); };
  const K ks[] = {{"loop (x + 0)", k_empty}, {"fma f64", k_fma}, {"mul f64", k_mul},
                  {"add f64", k_add}, {"a / x (IEEE div)", k_div}, {"divk (Markstein)", k_divk},
                  {"sqrt", k_sqrt}, {"rint", k_rint}, {"ocml sincos", k_ocml_sincos},
                  {"sincos_t", k_sincos_t}, {"ocml cos", k_ocml_cos}, {"cos_t", k_cos_t},
                  {"ocml atan2", k_ocml_atan2}, {"ocml pow(., 3.5)", k_pow_ocml},
                  {"pow_3p5", k_pow_3p5}, {"f64->f32->f64", k_cvt_f32},
                  {"select (cmp + cndmask)", k_select}, {"if/else uniform", k_branch},
                  {"if (never, heavy) + fma", k_branch_skip}, {"2x (if (never) + fma)", k_branch_skip2},
                  {"pymod360 (fast path)", k_pymod360},
                  {"if (expect 0) + fma", k_branch_expect}, {"if (ballot) + fma", k_branch_ballot},
                  {"if (__any) + fma", k_branch_any},
                  {"two nested selects", k_cmp_sel2},
                  {"pymod360_s (1 select)", k_pymod360_s}, {"pymod360_r (2 selects)", k_pymod360_r},
                  {"if (uniform SGPR) + fma", k_branch_uniform}};
  for (const K& k : ks) {
    long long best = 1LL << 62;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, din, dout, dc);
      long long c;
      (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
      if (c < best) best = c;
    }
    std::printf("%-22s %8.1f cycles per link\n", k.n, (double)best / ITER);
  }
  return 0;
}
