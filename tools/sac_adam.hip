// Adam step for the C5 learner (tools/sac_torch.py): every parameter tensor of one or more
// optimizer groups in ONE launch, one element per thread.
//
// torch's fused Adam (multi_tensor_apply) gives each workgroup a 65,536-element chunk, so the
// SAC learner's 67 k / 134 k-parameter groups run on a handful of workgroups, ~28 us per step
// each (profiles/r02/c5_kernel_stats.csv); here the same update runs on ~800 workgroups.
// Semantics of torch.optim.Adam (amsgrad=False, weight_decay=0, maximize=False), in fp32 as
// torch's opmath for fp32 parameters:
//   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2
//   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// with t read from device memory (the caller increments it once per update), so the launch
// can be captured in a HIP graph.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SAC_ADAM_MAX_TENSORS 16

extern "C" {
typedef struct {
  int32_t n;                                   // tensors in the table
  int32_t start[SAC_ADAM_MAX_TENSORS + 1];     // first workgroup of each tensor (prefix sums)
  int64_t numel[SAC_ADAM_MAX_TENSORS];
  float* p[SAC_ADAM_MAX_TENSORS];
  const float* g[SAC_ADAM_MAX_TENSORS];
  float* m[SAC_ADAM_MAX_TENSORS];
  float* v[SAC_ADAM_MAX_TENSORS];
} sac_adam_table;
}

namespace {

constexpr int BLOCK = 256;

__global__ __launch_bounds__(BLOCK) void adam_kernel(sac_adam_table T, const float* __restrict__ step,
                                                      float lr, float b1, float b2, float eps) {
  const int blk = blockIdx.x;
  int i = 0;
  while (i + 1 < T.n && blk >= T.start[i + 1]) ++i;   // <= 16 tensors: a short scan
  const int64_t k = (int64_t)(blk - T.start[i]) * BLOCK + threadIdx.x;
  if (k >= T.numel[i]) return;
  const float t = *step;
  const float bc1 = 1.0f - powf(b1, t);
  const float bc2 = 1.0f - powf(b2, t);
  const float g = T.g[i][k];
  const float m = b1 * T.m[i][k] + (1.0f - b1) * g;
  const float v = b2 * T.v[i][k] + (1.0f - b2) * g * g;
  T.m[i][k] = m;
  T.v[i][k] = v;
  const float denom = sqrtf(v) / sqrtf(bc2) + eps;
  T.p[i][k] -= (lr / bc1) * m / denom;
}

}  // namespace

extern "C" int32_t sac_adam_step(const sac_adam_table* T, const float* step, float lr, float b1,
                                 float b2, float eps, void* stream) {
  if (!T || !step || T->n < 1 || T->n > SAC_ADAM_MAX_TENSORS) return -1;
  for (int i = 0; i < T->n; ++i) {
    if (!T->p[i] || !T->g[i] || !T->m[i] || !T->v[i] || T->numel[i] <= 0) return -1;
    if (T->start[i + 1] - T->start[i] != (int32_t)((T->numel[i] + BLOCK - 1) / BLOCK)) return -1;
  }
  if (T->start[0] != 0) return -1;
  hipLaunchKernelGGL(adam_kernel, dim3(T->start[T->n]), dim3(BLOCK), 0, (hipStream_t)stream, *T,
                     step, lr, b1, b2, eps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
