// Probe on gfx950: bsg_fastmath.h's powers and Markstein divisions as the device computes
// them, against (a) the same code on the host (bit-identical expected: FMA/mul/add only),
// (b) glibc pow / IEEE '/' (what NumPy computes), (c) the device libm pow it replaces.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/probe/fastmath_probe.hip -o tools/probe/fastmath_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../bluesky-gym-hallucination_amd/csrc/bsg_fastmath.h"

constexpr int NF = 6;   // trop, 3.5, 2/7, division by 6371000, sin, cos on [-100, 100]
__global__ void k(const double* x, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = x[i];
  const double xt = 0.75 + 0.25 * a, x35 = 1.0 + 0.3 * a, x27 = 1.0 + a;
  out[(size_t)i * 2 * NF + 0] = bsg::pow_trop(xt);
  out[(size_t)i * 2 * NF + 1] = bsg::pow_3p5(x35);
  out[(size_t)i * 2 * NF + 2] = bsg::pow_2o7(x27);
  out[(size_t)i * 2 * NF + 3] = bsg::divk((a - 0.5) * 3e4, 6371000.0);
  const double xa = (a - 0.5) * 200.0;
  bsg::sincos_t(xa, &out[(size_t)i * 2 * NF + 4], &out[(size_t)i * 2 * NF + 5]);
  out[(size_t)i * 2 * NF + NF + 0] = pow(xt, 4.256848030018761);
  out[(size_t)i * 2 * NF + NF + 1] = pow(x35, 3.5);
  out[(size_t)i * 2 * NF + NF + 2] = pow(x27, 2.0 / 7.0);
  out[(size_t)i * 2 * NF + NF + 3] = ((a - 0.5) * 3e4) / 6371000.0;
  sincos(xa, &out[(size_t)i * 2 * NF + NF + 4], &out[(size_t)i * 2 * NF + NF + 5]);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), o((size_t)2 * NF * n);
  std::mt19937_64 rng(3);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (int i = 0; i < n; ++i) x[i] = U(rng);
  double *dx, *dout;
  if (hipMalloc(&dx, (size_t)n * 8) != hipSuccess || hipMalloc(&dout, o.size() * 8) != hipSuccess) return 1;
  (void)hipMemcpy(dx, x.data(), (size_t)n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
  (void)hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
  const char* name[NF] = {"pow(x, 4.2568..) x in [0.75, 1]", "pow(z, 3.5) z in [1, 1.3]",
                          "pow(y, 2/7) y in [1, 2]", "x / 6371000 (divk)",
                          "sin(x) x in [-100, 100]", "cos(x) x in [-100, 100]"};
  for (int f = 0; f < NF; ++f) {
    long host_diff = 0, ref_diff = 0, ocml_diff = 0;
    for (int i = 0; i < n; ++i) {
      const double a = x[i];
      const double xt = 0.75 + 0.25 * a, x35 = 1.0 + 0.3 * a, x27 = 1.0 + a;
      double host, ref;
      switch (f) {
        case 0: host = bsg::pow_trop(xt); ref = std::pow(xt, 4.256848030018761); break;
        case 1: host = bsg::pow_3p5(x35); ref = std::pow(x35, 3.5); break;
        case 2: host = bsg::pow_2o7(x27); ref = std::pow(x27, 2.0 / 7.0); break;
        case 3: {
          volatile double num = (a - 0.5) * 3e4, den = 6371000.0;
          host = bsg::divk((a - 0.5) * 3e4, 6371000.0); ref = num / den;
          break;
        }
        case 4: host = bsg::sin_t((a - 0.5) * 200.0); ref = std::sin((a - 0.5) * 200.0); break;
        default: host = bsg::cos_t((a - 0.5) * 200.0); ref = std::cos((a - 0.5) * 200.0);
      }
      const double dev = o[(size_t)i * 2 * NF + f], ocml = o[(size_t)i * 2 * NF + NF + f];
      host_diff += std::memcmp(&dev, &host, 8) != 0;
      ref_diff += std::memcmp(&dev, &ref, 8) != 0;
      ocml_diff += std::memcmp(&ocml, &ref, 8) != 0;
    }
    std::printf("%-34s device!=host-emulation %ld   device!=glibc/IEEE %ld (%.3f%%)   "
                "device-libm!=glibc/IEEE %ld (%.3f%%)   of %d\n",
                name[f], host_diff, ref_diff, 100.0 * ref_diff / n, ocml_diff, 100.0 * ocml_diff / n, n);
  }
  return 0;
}
