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
// 4096 envs is launch-bound, not arithmetic: 0.54 GFLOP).  Here: one workgroup of 512
// threads per 16 envs; a thread owns a hidden unit for 8 of the workgroup's rows, so each
// weight element is read once per workgroup (the 257 KB of weights stay in L2) and each
// LDS activation read is a wave-wide broadcast.  fp32 throughout (the MLP's dtype): the
// 256 x 256 layer on the matrix cores (f32-input MFMA, exact fp32 products, 16 x 16 tiles =
// the workgroup's 16 rows), the small first layer and the heads on the VALU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsg_internal.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int H = 256;       // hidden width (SB3 default net_arch for SAC)
constexpr int NT = 512;      // threads per workgroup: 8 waves, two per SIMD (hide the L2 latency of W1)
constexpr int R = 16;        // env rows per workgroup (= the MFMA tile's 16 rows)
constexpr int OMAX = 256;    // widest observation row handled
constexpr int AMAX = 4;      // widest action
constexpr int HS = H + 4;    // s_h row stride (16-B aligned rows, float4 reads spread over banks)
constexpr int XS = OMAX + 1; // s_x row stride (the heads read 4 rows per wave: no bank aliasing)

__global__ __launch_bounds__(NT) void sac_actor_kernel(bsg_sac_actor w, const float* __restrict__ obs,
                                                     int E, int ostride, const float* __restrict__ eps,
                                                     double* __restrict__ act, float* __restrict__ logp) {
  __shared__ float s_x[R * XS];     // observation rows, then layer-1 activations
  __shared__ float s_h[R * HS];     // layer-0 activations
  const int j = threadIdx.x;
  const int row0 = blockIdx.x * R;
  const int O = w.obs_dim, A = w.act_dim;
  const int nrow = min(R, E - row0);

  // stage the observation tile (rows past E read as 0; their outputs are never stored)
  for (int i = j; i < R * O; i += NT) {
    const int r = i / O, k = i - r * O;
    s_x[r * XS + k] = r < nrow ? obs[(size_t)(row0 + r) * ostride + k] : 0.0f;
  }
  __syncthreads();

  // layer 0: [R, O] x [O, H]; thread j owns hidden unit j % H for rows 8 (j / H) .. + 7
  {
    constexpr int RH = R * H / NT;
    const int col = j & (H - 1), rb = (j / H) * RH;
    float acc[RH];
    const float b = w.b0[col];
#pragma unroll
    for (int r = 0; r < RH; ++r) acc[r] = b;
    const float* wr = w.w0 + (size_t)col * O;
    for (int k = 0; k < O; ++k) {
      const float wk = wr[k];
#pragma unroll
      for (int r = 0; r < RH; ++r) acc[r] = __builtin_fmaf(s_x[(rb + r) * XS + k], wk, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < RH; ++r) s_h[(rb + r) * HS + col] = fmaxf(acc[r], 0.0f);
  }
  __syncthreads();
  // layer 1: [R, H] x [H, H] on the matrix cores (v_mfma_f32_16x16x4_f32: exact fp32
  // products, fp32 accumulation -- the VALU form of this loop was bound by the LDS broadcast
  // of the activations, one ds_read_b128 per 4 FMAs).  Wave v owns the output columns
  // [32v, 32v + 32) as two 16 x 16 tiles.  Lane l (m = l & 15, g = l >> 4) supplies
  // A[m][k] = h0[m][k] and B[k][n] = W1[n][k] for n = 32v + 16t + m; over a 16-wide k block
  // the lane's k slot g covers k0 + 4g .. k0 + 4g + 3 (one float4 of h0 from LDS, one float4
  // of W1's row n from L2), consumed one component per MFMA -- a permutation of the k sum.
  constexpr int TW = H / 16 / (NT / 64);   // tiles per wave
  f32x4 c[TW];
  {
    const int lane = j & 63, wv = j >> 6, m = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < TW; ++t) c[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const float* wrow = w.w1 + (size_t)(16 * TW * wv + m) * H + 4 * g;
#pragma unroll 4
    for (int k0 = 0; k0 < H; k0 += 16) {
      const float4 av = *reinterpret_cast<const float4*>(&s_h[m * HS + k0 + 4 * g]);
      float4 bv[TW];
#pragma unroll
      for (int t = 0; t < TW; ++t) bv[t] = *reinterpret_cast<const float4*>(wrow + (size_t)16 * t * H + k0);
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        c[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv[t].x, c[t], 0, 0, 0);
        c[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv[t].y, c[t], 0, 0, 0);
        c[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv[t].z, c[t], 0, 0, 0);
        c[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv[t].w, c[t], 0, 0, 0);
      }
    }
    // D[row = 4g + i][col = m] of tile t is h1 before bias/ReLU; s_x is free once layer 0
    // has read it (the barrier above)
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int n = 16 * TW * wv + 16 * t + m;
      const float b = w.b1[n];
#pragma unroll
      for (int i = 0; i < 4; ++i) s_x[(4 * g + i) * XS + n] = fmaxf(c[t][i] + b, 0.0f);
    }
  }
  __syncthreads();

  // heads (the first 256 threads): thread (r = j / 16, q = j % 16) sums k = q, q + 16, ... for each of the 2A outputs,
  // then the 16 lanes of the row reduce by xor-shuffles (all within one wave)
  if (j >= R * 16) return;
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
  hipLaunchKernelGGL(sac_actor_kernel, dim3(grid), dim3(NT), 0, stream, w, obs, E, ostride, eps,
                     act, logp);
  return hipGetLastError();
}

}  // namespace bsg
