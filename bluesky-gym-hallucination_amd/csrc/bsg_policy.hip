// Device policy: the SB3 SAC actor (MultiInputPolicy, net_arch [256, 256]) evaluated on the
// step kernel's fp32 observation rows as ONE fused HIP kernel, writing the fp64 action rows
// bsg_step reads.  It replaces, for a batch of E envs, what SB3 runs per vector step:
//   model.predict(obs, deterministic=True)            (reference main.py:54,
//                                                      scripts/multi_processing_example.py:70)
//   SAC.collect_rollouts -> actor.action_log_prob      (stable_baselines3 2.x sac/policies.py,
//                                                      Actor.forward / action_log_prob; the
//                                                      library is not vendored in the reference)
// i.e. latent = ReLU(W1 ReLU(W0 x + b0) + b1); mu = Wmu latent + bmu;
// log_std = clamp(Wls latent + bls, -20, 2); u = mu + exp(log_std) * eps; a = tanh(u);
// log_prob = sum_a [-eps^2/2 - log_std - log(2 pi)/2] - sum_a log(1 - a^2 + 1e-6).
//
// In torch that is ~25 kernels of 3-9 us each per vector step (the policy's whole cost at
// 4096 envs is launch-bound, not arithmetic: 0.54 GFLOP).  Here: one workgroup of 256
// threads per 16 envs; thread j owns hidden unit j for the workgroup's 16 rows, so each
// weight element is read once per workgroup (the 257 KB of weights stay in L2) and each
// LDS activation read is a wave-wide broadcast.  fp32 FMA throughout (the MLP's dtype);
// no MFMA: the batch-16 tile of a 256 x 256 layer is 1 M FMA per workgroup, below the
// launch cost it replaces.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsg_internal.h"

namespace {

constexpr int H = 256;       // hidden width (SB3 default net_arch for SAC)
constexpr int R = 16;        // env rows per workgroup
constexpr int OMAX = 256;    // widest observation row handled
constexpr int AMAX = 4;      // widest action
constexpr int XS = OMAX + 1; // s_x row stride (the heads read 4 rows per wave: no bank aliasing)

__global__ __launch_bounds__(H) void sac_actor_kernel(bsg_sac_actor w, const float* __restrict__ obs,
                                                     int E, int ostride, const float* __restrict__ eps,
                                                     double* __restrict__ act, float* __restrict__ logp) {
  __shared__ float s_x[R * XS];     // observation rows, then layer-1 activations
  __shared__ float s_h[R * H];      // layer-0 activations
  const int j = threadIdx.x;
  const int row0 = blockIdx.x * R;
  const int O = w.obs_dim, A = w.act_dim;
  const int nrow = min(R, E - row0);

  // stage the observation tile (rows past E read as 0; their outputs are never stored)
  for (int i = j; i < R * O; i += H) {
    const int r = i / O, k = i - r * O;
    s_x[r * XS + k] = r < nrow ? obs[(size_t)(row0 + r) * ostride + k] : 0.0f;
  }
  __syncthreads();

  float acc[R];
  // layer 0: [R, O] x [O, H]
  {
    const float b = w.b0[j];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = b;
    const float* wr = w.w0 + (size_t)j * O;
    for (int k = 0; k < O; ++k) {
      const float wk = wr[k];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = __builtin_fmaf(s_x[r * XS + k], wk, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) s_h[r * H + j] = fmaxf(acc[r], 0.0f);
  }
  __syncthreads();
  // layer 1: [R, H] x [H, H]; weight row j (nn.Linear [out, in]) read as float4 along k
  {
    const float b = w.b1[j];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = b;
    const float4* wr = reinterpret_cast<const float4*>(w.w1 + (size_t)j * H);
#pragma unroll 4
    for (int k4 = 0; k4 < H / 4; ++k4) {
      const float4 wk = wr[k4];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float4 x = *reinterpret_cast<const float4*>(&s_h[r * H + 4 * k4]);
        float a = acc[r];
        a = __builtin_fmaf(x.x, wk.x, a);
        a = __builtin_fmaf(x.y, wk.y, a);
        a = __builtin_fmaf(x.z, wk.z, a);
        a = __builtin_fmaf(x.w, wk.w, a);
        acc[r] = a;
      }
    }
  }
  // s_x is free once layer 0 has read it (the barrier above): layer-1 activations go there
#pragma unroll
  for (int r = 0; r < R; ++r) s_x[r * XS + j] = fmaxf(acc[r], 0.0f);
  __syncthreads();

  // heads: thread (r = j / 16, q = j % 16) sums k = q, q + 16, ... for each of the 2A outputs,
  // then the 16 lanes of the row reduce by xor-shuffles (all within one wave)
  const int r = j >> 4, q = j & 15;
  float out[2 * AMAX];
#pragma unroll
  for (int o = 0; o < 2 * AMAX; ++o) {
    float s = 0.0f;
    if (o < 2 * A) {
      const float* wo = o < A ? w.w_mu + (size_t)o * H : w.w_ls + (size_t)(o - A) * H;
#pragma unroll 4
      for (int i = 0; i < H / 16; ++i) {
        const int k = q + 16 * i;
        s = __builtin_fmaf(s_x[r * XS + k], wo[k], s);
      }
    }
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) s += __shfl_xor(s, m, 16);
    out[o] = s;
  }
  if (q != 0 || r >= nrow) return;
  const size_t row = (size_t)row0 + r;
  float lp = 0.0f;
  for (int a = 0; a < A; ++a) {
    const float mu = out[a] + w.b_mu[a];
    const float ls = fminf(fmaxf(out[A + a] + w.b_ls[a], -20.0f), 2.0f);
    const float e = eps ? eps[row * A + a] : 0.0f;
    const float u = eps ? __builtin_fmaf(expf(ls), e, mu) : mu;
    const float ta = tanhf(u);
    act[row * A + a] = (double)ta;
    lp += -0.5f * e * e - ls - 0.91893853320467274f - logf(1.0f - ta * ta + 1e-6f);
  }
  if (logp) logp[row] = lp;
}

}  // namespace

namespace bsg {

// Shapes and pointers are validated by bsg_policy_sac (bsg_abi.cpp).
hipError_t launch_sac_actor(const bsg_sac_actor& w, const float* obs, int E, int ostride,
                            const float* eps, double* act, float* logp, hipStream_t stream) {
  const int grid = (E + R - 1) / R;
  hipLaunchKernelGGL(sac_actor_kernel, dim3(grid), dim3(H), 0, stream, w, obs, E, ostride, eps,
                     act, logp);
  return hipGetLastError();
}

}  // namespace bsg
