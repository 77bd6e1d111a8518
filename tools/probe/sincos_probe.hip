// Probe: is ocml sincos() bit-identical to separate sin()/cos()?  And fmod-based pymod.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>
__global__ void k(const double* x, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s, c;
  sincos(x[i], &s, &c);
  out[4 * i + 0] = s - sin(x[i]) == 0 ? 0.0 : 1.0;
  out[4 * i + 1] = c - cos(x[i]) == 0 ? 0.0 : 1.0;
  double a = x[i] * 1000.0, b = 360.0;
  double mod = fmod(a, b);
  if (mod != 0.0) { if ((b < 0.0) != (mod < 0.0)) mod += b; } else mod = copysign(0.0, b);
  out[4 * i + 2] = mod;
  out[4 * i + 3] = pow(x[i] * x[i] + 1.0, 3.5);
}
int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), o(4 * n);
  srand(1);
  for (int i = 0; i < n; ++i) x[i] = ((double)rand() / RAND_MAX - 0.5) * 20.0;
  double *dx, *dout;
  (void)hipMalloc(&dx, n * 8); (void)hipMalloc(&dout, 4 * n * 8);
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
  (void)hipMemcpy(o.data(), dout, 4 * n * 8, hipMemcpyDeviceToHost);
  long bs = 0, bc = 0, bm = 0, bp = 0;
  for (int i = 0; i < n; ++i) {
    bs += o[4 * i] != 0; bc += o[4 * i + 1] != 0;
    double a = x[i] * 1000.0, ref = std::fmod(a, 360.0);
    if (ref != 0.0) { if ((ref < 0.0) != (360.0 < 0.0)) ref += 360.0; } else ref = std::copysign(0.0, 360.0);
    bm += std::memcmp(&ref, &o[4 * i + 2], 8) != 0;
    double pr = std::pow(x[i] * x[i] + 1.0, 3.5);
    bp += std::memcmp(&pr, &o[4 * i + 3], 8) != 0;
  }
  printf("sincos!=sin %ld  sincos!=cos %ld  pymod!=host %ld  pow!=glibc %ld  (of %d)\n", bs, bc, bm, bp, n);
  return 0;
}
