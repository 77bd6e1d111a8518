// The C5 learner's SAC update with its elementwise work fused (tools/sac_torch.py FusedSAC).
//
// SB3's SAC update (scripts/descent_env_sac.py:25-34 -> SB3 2.x SAC.train, one gradient step)
// at batch 256 through 256-wide MLPs is ~100 small kernels as torch autograd runs it
// (bias copies, ReLU and its backward, bias-gradient reductions, the loss terms and the
// squashed Gaussian as separate launches), each paying the ~1.5 us dependent-kernel boundary
// (MI355X_MICROARCH.md 'boundary').  FusedSAC writes the forward and backward passes out; the
// 256 x 256 products are gemm256_kernel launches (below; rocBLAS with SAC_GEMM=blas); everything
// between two GEMMs is one of the kernels below, so an update is 19 launches:
//
//   in_layer     relu(x W + b) for a layer whose K is the observation (+ action) width
//   in_layer_pair  the actor's and the online critics' first layers in one launch
//   noise_sample the update's uniforms and normals (and the next action sample's), Philox,
//                then the replay rows the uniforms draw and the Adam step-count tick
//   actor_head   h1 = relu(p1 + b1), mu / log_std heads, SB3's squashed Gaussian (a, logp),
//                and on the next-observation rows the target critics' first layer
//   critic_head  g1 = relu(p1 + b1), q = g1 w2 + b2 for both critics, then per mode the TD
//                target y, the twin-MSE gradient dq, or the actor loss's dq / dlogp
//   td_critic_head  the target critics and the online critics of one [4, B, H] product: y,
//                then the online heads' dq (one launch for both)
//   (the heads' backward, dg1 = dq w2 (g1 > 0), in td_critic_head / critic_head's launch)
//   critic_bwd_in     the first layer's gradients from dg0 (g0 > 0), and the w2 / b2 / b1
//                     gradients (column sums)
//   actor_bwd_head    the critics' action gradient, the squashed Gaussian's backward and
//                     dh1 = (dmu Wmu + dlsr Wls)(h1 > 0)
//   actor_bwd_in      the first layer's gradients from dh0 (h0 > 0), then the heads' and b1's
//                     gradients and d log_alpha (column sums, actor_cols)
//   (SB3's polyak_update of the target critics runs inside the critic's Adam launch,
//   tools/sac_adam.hip sac_adam_step_polyak)
//
// Layouts: the actor's torch Linear weights ([out, in]); the twin critics stacked as
// tools/sac_torch.py TwinQ keeps them (w0 [2, in, H], w1 [2, H, H], w2 [2, H, 1]).  H = 256.
// Every column sum runs over 16 row groups in row order and adds them in group order:
// deterministic.  fp32,
// -ffp-contract=off; results agree with the autograd path to fp32 rounding (the association
// of the sums differs), checked by tests/test_gpu_sac_adam.py.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace {

constexpr int H = 256;
constexpr float LOG_SQRT_2PI = 0.91893853320467274f;

__device__ __forceinline__ float wave_sum(float v) {
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// out[c][r][u] = relu(b[c][u] + sum_k x[r][k] w[c][k][u])   (w_ku: critic layout [c][k][u])
// or             relu(b[u] + sum_k x[r][k] w[u][k])         (!w_ku: torch Linear [u][k], c = 0)
// x[r] = [xa row (Ka) | xb row (Kb)]; rows r >= split read xa_hi instead of xa.
__global__ __launch_bounds__(256) void in_layer_kernel(
    const float* __restrict__ xa, const float* __restrict__ xa_hi, int split, int lda, int Ka,
    const float* __restrict__ xb, int ldb, int Kb, int R, int nC, const float* __restrict__ w,
    int w_ku, const float* __restrict__ b, float* __restrict__ out) {
  const int u = threadIdx.x;
  const int r = blockIdx.x;
  const int c = blockIdx.y;
  if (r >= R || c >= nC) return;
  const float* xr = r < split ? xa + (size_t)r * lda : xa_hi + (size_t)(r - split) * lda;
  const int K = Ka + Kb;
  float acc = 0.0f;
  for (int k0 = 0; k0 < K; k0 += 8) {       // (each chunk's loads issued before its FMAs)
    float xv[8], wv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int k = min(k0 + t, K - 1);
      xv[t] = k < Ka ? xr[k] : xb[(size_t)r * ldb + (k - Ka)];
      wv[t] = w_ku ? w[((size_t)c * K + k) * H + u] : w[(size_t)u * K + k];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t)
      if (k0 + t < K) acc += xv[t] * wv[t];
  }
  const float z = acc + b[(size_t)c * H + u];
  out[((size_t)c * R + r) * H + u] = z > 0.0f ? z : 0.0f;
}

// two first layers in one launch: blockIdx.y == 0 the actor's (rows xa / xa_hi, torch
// Linear layout), y = 1, 2 the online critics' on [ya | yb] (rows < R2, critic layout) --
// in_layer's sums, k in order
__global__ __launch_bounds__(256) void in_layer_pair_kernel(
    const float* __restrict__ xa, const float* __restrict__ xa_hi, int split, int lda, int Ka,
    int R1, const float* __restrict__ w1, const float* __restrict__ b1, float* __restrict__ out1,
    const float* __restrict__ ya, int ldya, int Kya, const float* __restrict__ yb, int ldyb,
    int Kyb, int R2, const float* __restrict__ w2, const float* __restrict__ b2,
    float* __restrict__ out2) {
  const int u = threadIdx.x;
  const int r = blockIdx.x;
  if (blockIdx.y == 0) {
    if (r >= R1) return;
    const float* xr = r < split ? xa + (size_t)r * lda : xa_hi + (size_t)(r - split) * lda;
    float acc = 0.0f;
    for (int k0 = 0; k0 < Ka; k0 += 8) {
      float xv[8], wv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int k = min(k0 + t, Ka - 1);
        xv[t] = xr[k];
        wv[t] = w1[(size_t)u * Ka + k];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (k0 + t < Ka) acc += xv[t] * wv[t];
    }
    const float z = acc + b1[u];
    out1[(size_t)r * H + u] = z > 0.0f ? z : 0.0f;
  } else {
    const int c = blockIdx.y - 1;
    if (r >= R2) return;
    const int K = Kya + Kyb;
    float acc = 0.0f;
    for (int k0 = 0; k0 < K; k0 += 8) {
      float xv[8], wv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int k = min(k0 + t, K - 1);
        xv[t] = k < Kya ? ya[(size_t)r * ldya + k] : yb[(size_t)r * ldyb + (k - Kya)];
        wv[t] = w2[((size_t)c * K + k) * H + u];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t)
        if (k0 + t < K) acc += xv[t] * wv[t];
    }
    const float z = acc + b2[(size_t)c * H + u];
    out2[((size_t)c * R2 + r) * H + u] = z > 0.0f ? z : 0.0f;
  }
}

// the update's random numbers in one launch, Philox4x32-10 (Salmon et al. 2011) keyed by
// seed, counter = (launch number, element): u ~ U[0, 1) for the replay sample, the squashed
// Gaussian's eps ~ N(0, 1) (Box-Muller) for the update and for the next vector step's action
// sample.  One workgroup; its thread 0 advances the launch number after every thread has
// read it, so replays of a captured graph draw new numbers.
__device__ __forceinline__ void philox10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

__global__ __launch_bounds__(1024) void noise_kernel(unsigned long long* __restrict__ launch,
                                                     unsigned long long seed,
                                                     float* __restrict__ u, int nu,
                                                     float* __restrict__ e1, int n1,
                                                     float* __restrict__ e2, int n2) {
  const unsigned long long L = launch[0];
  const int total = nu + n1 + n2;
  for (int i = threadIdx.x; 2 * i < total + 1; i += blockDim.x) {
    uint32_t c[4] = {(uint32_t)L, (uint32_t)(L >> 32), (uint32_t)i, 0x53414331u};
    philox10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    // two outputs per counter: uniforms from c[0], c[1]; normals from (c[0], c[1]) and
    // (c[2], c[3]) by Box-Muller
    const float v1 = 1.0f - u01(c[0]), v2 = u01(c[1]);
    const float v3 = 1.0f - u01(c[2]), v4 = u01(c[3]);
    const float g1 = sqrtf(-2.0f * logf(v1)) * cospif(2.0f * v2);
    const float g2 = sqrtf(-2.0f * logf(v3)) * cospif(2.0f * v4);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = 2 * i + h;
      if (o < nu) u[o] = h == 0 ? u01(c[0]) : u01(c[1]);
      else if (o < nu + n1) e1[o - nu] = h == 0 ? g1 : g2;
      else if (o < total) e2[o - nu - n1] = h == 0 ? g1 : g2;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) launch[0] = L + 1;
}

// noise_kernel followed, in the same workgroup, by the replay sample those uniforms draw
// (sac_adam.hip replay_sample_kernel's index arithmetic: idx = min(int(u * size), cap - 1))
// and the optimizers' step-count tick -- the update's first three launches in one
__global__ __launch_bounds__(1024) void noise_sample_kernel(
    unsigned long long* __restrict__ launch, unsigned long long seed, float* __restrict__ u, int nu,
    float* __restrict__ e1, int n1, float* __restrict__ e2, int n2, const float* __restrict__ buf,
    long long cap, int W, const long long* __restrict__ size, float* __restrict__ rows,
    float* __restrict__ step) {
  __shared__ float us[1024];
  const unsigned long long L = launch[0];
  const int total = nu + n1 + n2;
  for (int i = threadIdx.x; 2 * i < total + 1; i += blockDim.x) {
    uint32_t c[4] = {(uint32_t)L, (uint32_t)(L >> 32), (uint32_t)i, 0x53414331u};
    philox10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float v1 = 1.0f - u01(c[0]), v2 = u01(c[1]);
    const float v3 = 1.0f - u01(c[2]), v4 = u01(c[3]);
    const float g1 = sqrtf(-2.0f * logf(v1)) * cospif(2.0f * v2);
    const float g2 = sqrtf(-2.0f * logf(v3)) * cospif(2.0f * v4);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = 2 * i + h;
      if (o < nu) {
        const float uv = h == 0 ? u01(c[0]) : u01(c[1]);
        u[o] = uv;
        us[o] = uv;
      } else if (o < nu + n1) {
        e1[o - nu] = h == 0 ? g1 : g2;
      } else if (o < total) {
        e2[o - nu - n1] = h == 0 ? g1 : g2;
      }
    }
  }
  __syncthreads();
  const long long sz = size[0];
  for (long long i = threadIdx.x; i < (long long)nu * W; i += blockDim.x) {
    const int b = (int)(i / W), col = (int)(i - (long long)b * W);
    long long idx = (long long)(us[b] * (float)sz);
    if (idx > cap - 1) idx = cap - 1;
    rows[i] = buf[(size_t)idx * W + col];
  }
  if (threadIdx.x == 0) {
    launch[0] = L + 1;
    step[0] += 1.0f;                         // HipAdam.tick (t.add_(1.0)): read only after this launch
  }
}

// one wave per row: h1 = relu(p1 + b1); mu = h1 Wmu^T + bmu; lsr = h1 Wls^T + bls;
// SB3's squashed Gaussian (sac_adam.hip sq_gauss_fwd_kernel): a = tanh(mu + exp(clamp(lsr)) eps)
__global__ __launch_bounds__(256) void actor_head_kernel(
    const float* __restrict__ p1, const float* __restrict__ b1, const float* __restrict__ wmu,
    const float* __restrict__ bmu, const float* __restrict__ wls, const float* __restrict__ bls,
    const float* __restrict__ eps, int R, int A, float* __restrict__ h1, float* __restrict__ mu,
    float* __restrict__ lsr, float* __restrict__ a_out, float* __restrict__ logp,
    int RT, const float* __restrict__ xt, int ldxt, int Kxt, const float* __restrict__ tw0,
    const float* __restrict__ tb0, float* __restrict__ g0t) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  float av[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float hv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = lane + 64 * i;
    const float z = p1[(size_t)r * H + u] + b1[u];
    hv[i] = z > 0.0f ? z : 0.0f;
    h1[(size_t)r * H + u] = hv[i];
  }
  float s1 = 0.0f, s2 = 0.0f;
  for (int j = 0; j < A; ++j) {
    float pm = 0.0f, pl = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = lane + 64 * i;
      pm += hv[i] * wmu[(size_t)j * H + u];
      pl += hv[i] * wls[(size_t)j * H + u];
    }
    const float m = wave_sum(pm) + bmu[j];
    const float lr_ = wave_sum(pl) + bls[j];
    const int ij = r * A + j;
    const float ls = fminf(fmaxf(lr_, -20.0f), 2.0f);
    const float sd = expf(ls);
    const float uu = m + sd * eps[ij];
    const float a = tanhf(uu);
    const float z = (uu - m) / sd;
    s1 += -0.5f * (z * z) - ls - LOG_SQRT_2PI;
    s2 += logf(1.0f - a * a + 1e-6f);
    av[j & 3] = a;
    if (lane == 0) {
      mu[ij] = m;
      lsr[ij] = lr_;
      a_out[ij] = a;
    }
  }
  if (lane == 0) logp[r] = s1 - s2;
  // rows r < RT (the next observations): the target critics' first layer on [x_r, a_r]
  // (in_layer's sum, k in order), so the TD target needs no launch of its own
  if (g0t && r < RT) {
    // (k in chunks of 8 with every load of a chunk issued before its FMAs: a k-at-a-time loop
    // paid one memory round trip per k; the sums run over k in order either way)
    const int K = Kxt + A;
    float acc[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[c][i] = 0.0f;
    for (int k0 = 0; k0 < K; k0 += 8) {
      float xv[8], wv[2][4][8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int k = min(k0 + t, K - 1);
        xv[t] = k < Kxt ? xt[(size_t)r * ldxt + k] : av[(k - Kxt) & 3];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i) wv[c][i][t] = tw0[((size_t)c * K + k) * H + lane + 64 * i];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (k0 + t < K) {
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[c][i] += xv[t] * wv[c][i][t];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = lane + 64 * i;
        const float z = acc[c][i] + tb0[(size_t)c * H + u];
        g0t[((size_t)c * RT + r) * H + u] = z > 0.0f ? z : 0.0f;
      }
    }
  }
}

enum { HEAD_TARGET = 0, HEAD_CRITIC = 1, HEAD_ACTOR_LOSS = 2, HEAD_TD_CRITIC = 3 };

// one wave per row, both critics: g1 = relu(p1 + b1) (stored unless TARGET), q = g1 w2 + b2.
//  TARGET:     y[r] = rew + gamma (1 - done) (min_c q - alpha logp2[r])      (sac_td_target)
//  CRITIC:     dq[c][r] = (1 / B) (2 (q - y[r])); lossp[r] = sum_c (q - y)^2 / B
//  ACTOR_LOSS: dlogp[r] = alpha / B; dq on the smaller critic -1 / B (split on a tie);
//              lossp[r] = (alpha logp[r] - min_c q) / B                          (sac_actor_loss)
__global__ __launch_bounds__(256) void critic_head_kernel(
    const float* __restrict__ p1, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, int B, int mode, const float* __restrict__ rows, int W,
    int col_r, int col_d, float gamma, const float* __restrict__ log_alpha,
    const float* __restrict__ logp, float* __restrict__ y, float* __restrict__ g1,
    float* __restrict__ q_out, float* __restrict__ dq, float* __restrict__ dlogp,
    float* __restrict__ lossp, float* __restrict__ dg1) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  float q[2], gk[2][4];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float part = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = lane + 64 * i;
      const size_t o = ((size_t)c * B + r) * H + u;
      const float z = p1[o] + b1[(size_t)c * H + u];
      const float g = z > 0.0f ? z : 0.0f;
      if (mode != HEAD_TARGET && g1) g1[o] = g;
      gk[c][i] = g;
      part += g * w2[(size_t)c * H + u];
    }
    q[c] = wave_sum(part) + b2[c];
  }
  if (mode == HEAD_ACTOR_LOSS && dg1) {
    // the actor loss's gradient through the critics' head (dg1), from the
    // row's dq -- wave-uniform, as lane 0 stores it below
    const float ng = -(1.0f / (float)B);
    const float mn = fminf(q[0], q[1]);
    float dqv[2];
    if (q[0] == q[1]) {
      dqv[0] = ng / 2.0f;
      dqv[1] = ng / 2.0f;
    } else {
      dqv[0] = q[0] == mn ? ng : 0.0f;
      dqv[1] = q[1] == mn ? ng : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = lane + 64 * i;
        dg1[((size_t)c * B + r) * H + u] = gk[c][i] > 0.0f ? dqv[c] * w2[(size_t)c * H + u] : 0.0f;
      }
    }
  }
  if (lane != 0) return;
  const float alpha = expf(log_alpha[0]);
  q_out[r] = q[0];
  q_out[B + r] = q[1];
  const float invB = 1.0f / (float)B;
  if (mode == HEAD_TARGET) {
    const float mn = fminf(q[0], q[1]);
    const float qt = mn - alpha * logp[r];
    const float d = rows[(size_t)r * W + col_d];
    const float rw = rows[(size_t)r * W + col_r];
    y[r] = rw + (gamma * (1.0f - d)) * qt;
  } else if (mode == HEAD_CRITIC) {
    float l = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float df = q[c] - y[r];
      dq[(size_t)c * B + r] = invB * (2.0f * df);
      l += df * df / (float)B;
    }
    lossp[r] = l;
  } else {
    const float gb = invB;
    dlogp[r] = gb * alpha;
    const float mn = fminf(q[0], q[1]);
    const float ng = -gb;
    if (q[0] == q[1]) {
      dq[r] = ng / 2.0f;
      dq[B + r] = ng / 2.0f;
    } else {
      dq[r] = q[0] == mn ? ng : 0.0f;
      dq[B + r] = q[1] == mn ? ng : 0.0f;
    }
    lossp[r] = (alpha * logp[r] - mn) / (float)B;
  }
}

// one wave per row, the target critics and the online critics of one [4, B, H] product (p1[0:2]
// the targets' on [o2, a2], p1[2:4] the online critics' on [o, a]): the TD target y (as
// HEAD_TARGET), then the online heads' g1 (stored, [2, B, H]), q and the twin-MSE gradient dq
// and loss terms (as HEAD_CRITIC) -- both heads in one launch
__global__ __launch_bounds__(256) void td_critic_head_kernel(
    const float* __restrict__ p1, const float* __restrict__ tb1, const float* __restrict__ tw2,
    const float* __restrict__ tb2, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, int B, const float* __restrict__ rows, int W, int col_r,
    int col_d, float gamma, const float* __restrict__ log_alpha, const float* __restrict__ logp,
    float* __restrict__ y, float* __restrict__ g1, float* __restrict__ q_out,
    float* __restrict__ dq, float* __restrict__ lossp, float* __restrict__ dg1) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  float q[4], gk[2][4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int cc = c & 1;
    const float* bb = c < 2 ? tb1 : b1;
    const float* ww = c < 2 ? tw2 : w2;
    float part = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = lane + 64 * i;
      const float z = p1[((size_t)c * B + r) * H + u] + bb[(size_t)cc * H + u];
      const float g = z > 0.0f ? z : 0.0f;
      if (c >= 2) {
        g1[((size_t)cc * B + r) * H + u] = g;
        gk[cc][i] = g;
      }
      part += g * ww[(size_t)cc * H + u];
    }
    q[c] = wave_sum(part) + (c < 2 ? tb2 : b2)[cc];
  }
  // (the row's scalars are wave-uniform: every lane evaluates them, lane 0 stores them)
  const float alpha = expf(log_alpha[0]);
  const float mn = fminf(q[0], q[1]);
  const float qt = mn - alpha * logp[r];
  const float d = rows[(size_t)r * W + col_d];
  const float rw = rows[(size_t)r * W + col_r];
  const float yr = rw + (gamma * (1.0f - d)) * qt;
  const float invB = 1.0f / (float)B;
  float dqv[2], l = 0.0f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float df = q[2 + c] - yr;
    dqv[c] = invB * (2.0f * df);
    l += df * df / (float)B;
  }
  // the critics' backward through their head (dg1 = dq w2 (g1 > 0))
  if (dg1) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = lane + 64 * i;
        dg1[((size_t)c * B + r) * H + u] = gk[c][i] > 0.0f ? dqv[c] * w2[(size_t)c * H + u] : 0.0f;
      }
    }
  }
  if (lane != 0) return;
  y[r] = yr;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    q_out[(size_t)c * B + r] = q[2 + c];
    dq[(size_t)c * B + r] = dqv[c];
  }
  lossp[r] = l;
}

// The column-sum kernels below: a workgroup of 256 threads takes 16 columns (blockIdx.x) of
// one critic (blockIdx.y) and splits the rows into 16 groups (threadIdx.x / 16); each thread
// loads its group's rows (16 at B = 256) up front, sums them in row order, and the 16
// partials are added in group order through LDS -- deterministic, every load of a thread in
// flight at once, and 16-32 workgroups instead of a few long serial loops (a one-thread-per-
// column loop over 256 rows took 25-45 us: profiles/r05/c5_kernel_stats_before.csv).
constexpr int NRG = 16;           // row groups per workgroup
constexpr int CPB = 16;           // columns per workgroup
constexpr int RPG = 16;           // rows per group held in registers at once

// combine the row groups' partials of NV values per column (in group order)
template <int NV>
__device__ __forceinline__ void group_sum(float (&v)[NV], float (*lds)[NRG][CPB]) {
  const int col = threadIdx.x % CPB, grp = threadIdx.x / CPB;
#pragma unroll
  for (int i = 0; i < NV; ++i) lds[i][grp][col] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float t = 0.0f;
#pragma unroll
    for (int q = 0; q < NRG; ++q) t += lds[i][q][col];
    v[i] = t;
  }
  __syncthreads();
}

__device__ __forceinline__ void group_rows(int R, int& r0, int& r1) {
  const int per = (R + NRG - 1) / NRG;
  r0 = (int)(threadIdx.x / CPB) * per;
  r1 = min(R, r0 + per);
}

// m = dg0 (g0 > 0); dw0[c][k][u] = sum_r x[r][k] m, db0[c][u] = sum_r m;  x[r] = [xa | xb].
// The rows' inputs x (shared by the workgroup's 16 columns) are staged in LDS once, so a
// thread loads only its rows' dg0 / g0 (the sums and their order are unchanged).
constexpr int kXR = 256, kXK = 48;       // staged rows / inputs (checked by the launchers)
// g1 != nullptr: also the head's column sums, dw2[c][u] = sum_r g1 dq,
// db1[c][u] = sum_r dq w2 (g1 > 0), db2[c] = sum_r dq (the same rows, order and groups)
__global__ __launch_bounds__(256) void critic_bwd_in_kernel(
    const float* __restrict__ dg0, const float* __restrict__ g0, const float* __restrict__ xa,
    int lda, int Ka, const float* __restrict__ xb, int ldb, int Kb, int B,
    float* __restrict__ dw0, float* __restrict__ db0, const float* __restrict__ g1,
    const float* __restrict__ dq, const float* __restrict__ w2, float* __restrict__ dw2,
    float* __restrict__ db1, float* __restrict__ db2) {
  __shared__ float lds[9][NRG][CPB];
  __shared__ float xl[kXR][kXK + 1];
  const int u = blockIdx.x * CPB + threadIdx.x % CPB;
  const int c = blockIdx.y;
  int r0, r1;
  group_rows(B, r0, r1);
  const int K = Ka + Kb;
  if (g1) {
    const float wv = w2[(size_t)c * H + u];
    float gg[RPG], dd[RPG];
#pragma unroll
    for (int t = 0; t < RPG; ++t) {
      const int r = min(r0 + t, r1 - 1);
      gg[t] = g1[((size_t)c * B + r) * H + u];
      dd[t] = dq[(size_t)c * B + r];
    }
    float v[3] = {0.0f, 0.0f, 0.0f};          // sum g1 dq, sum dg1, sum dq
#pragma unroll
    for (int t = 0; t < RPG; ++t) {
      if (r0 + t < r1) {
        const float val = gg[t] > 0.0f ? dd[t] * wv : 0.0f;
        v[0] += gg[t] * dd[t];
        v[1] += val;
        v[2] += dd[t];
      }
    }
    group_sum<3>(v, lds);
    if (threadIdx.x < CPB) {
      dw2[(size_t)c * H + u] = v[0];
      db1[(size_t)c * H + u] = v[1];
      if (u == 0) db2[c] = v[2];
    }
  }
  for (int q = threadIdx.x; q < B * K; q += blockDim.x) {
    const int r = q / K, k = q - r * K;
    xl[r][k] = k < Ka ? xa[(size_t)r * lda + k] : xb[(size_t)r * ldb + (k - Ka)];
  }
  float mm[RPG];
#pragma unroll
  for (int t = 0; t < RPG; ++t) {
    const int r = min(r0 + t, r1 - 1);
    const size_t o = ((size_t)c * B + r) * H + u;
    const float g = g0[o], d = dg0[o];
    mm[t] = (r0 + t < r1 && g > 0.0f) ? d : 0.0f;
  }
  __syncthreads();
  for (int k0 = 0; k0 < K; k0 += 8) {
    float v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // 8 weight sums, the bias sum
#pragma unroll
    for (int t = 0; t < RPG; ++t) {
      const int r = min(r0 + t, r1 - 1);
      v[8] += mm[t];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += xl[r][min(k0 + i, K - 1)] * mm[t];
    }
    group_sum<9>(v, lds);
    if (threadIdx.x < CPB) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (k0 + i < K) dw0[((size_t)c * K + k0 + i) * H + u] = v[i];
      if (k0 == 0) db0[(size_t)c * H + u] = v[8];
    }
  }
}

// one wave per row: dx[r][j] = sum_c sum_u w0[c][Ka + j][u] (dg0 (g0 > 0))[c][r][u], the
// gradient w.r.t. the critics' action inputs (columns Ka.. of their input)
// one wave per row: the squashed Gaussian's backward (sac_adam.hip sq_gauss_bwd_kernel) from
// (ga = dx, gl = dlogp), then dh1[r][u] = (sum_j dmu Wmu[j][u] + dlsr Wls[j][u]) (h1 > 0)
// ga == nullptr: the action gradient is the critics' (the sum over both critics of
// w0's action rows times dg0 (g0 > 0), computed here -- one launch less)
__global__ __launch_bounds__(256) void actor_bwd_head_kernel(
    const float* __restrict__ ga, const float* __restrict__ gl, const float* __restrict__ mu,
    const float* __restrict__ lsr, const float* __restrict__ eps, const float* __restrict__ a_out,
    const float* __restrict__ h1, const float* __restrict__ wmu, const float* __restrict__ wls,
    int R, int A, float* __restrict__ dmu, float* __restrict__ dlsr, float* __restrict__ dh1,
    const float* __restrict__ dg0, const float* __restrict__ g0, const float* __restrict__ w0,
    int K, int Ka) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const float g = gl[r];
  for (int j = 0; j < A; ++j) {
    const int i = r * A + j;
    float gaj;
    if (ga) {
      gaj = ga[i];
    } else {
      float part = 0.0f;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int uu = lane + 64 * t;
          const size_t o = ((size_t)c * R + r) * H + uu;
          const float m = g0[o] > 0.0f ? dg0[o] : 0.0f;
          part += w0[((size_t)c * K + Ka + j) * H + uu] * m;
        }
      }
      gaj = wave_sum(part);
    }
    const float x = lsr[i];
    const float ls = fminf(fmaxf(x, -20.0f), 2.0f);
    const float sd = expf(ls);
    const float u = mu[i] + sd * eps[i];
    const float z = (u - mu[i]) / sd;
    const float a = a_out[i];
    const float da = 1.0f - a * a;
    const float gu = gaj * da + g * (-z / sd + (2.0f * a / (da + 1e-6f)) * da);
    const float gm = gu + g * z / sd;
    const float gsd = gu * eps[i] + g * (z * z) / sd;
    const float gls = (x >= -20.0f && x <= 2.0f) ? gsd * sd - g : 0.0f;
    if (lane == 0) {
      dmu[i] = gm;
      dlsr[i] = gls;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int uu = lane + 64 * t;
      acc[t] += gm * wmu[(size_t)j * H + uu] + gls * wls[(size_t)j * H + uu];
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int uu = lane + 64 * t;
    dh1[(size_t)r * H + uu] = h1[(size_t)r * H + uu] > 0.0f ? acc[t] : 0.0f;
  }
}

// dWmu[j][u] = sum_r dmu[r][j] h1[r][u], dWls likewise, db1[u] = sum_r dh1 (per column, row
// groups as above); workgroup 0's waves 1-3 reduce the per-row terms, 4 rows per lane and a
// fixed shuffle tree: dbmu[j], dbls[j] and d log_alpha = -mean_r(logp + target_entropy) (SB3's
// ent_coef_loss = -(log_alpha * (logp + target_entropy).detach()).mean())
__device__ __forceinline__ void actor_cols(
    const float* __restrict__ dmu, const float* __restrict__ dlsr, const float* __restrict__ h1,
    const float* __restrict__ dh1, const float* __restrict__ logp, float target_entropy, int R,
    int A, float* __restrict__ dwmu, float* __restrict__ dwls, float* __restrict__ db1,
    float* __restrict__ dbmu, float* __restrict__ dbls, float* __restrict__ dlog_alpha,
    float (*lds)[NRG][CPB]) {
  const int u = blockIdx.x * CPB + threadIdx.x % CPB;
  int r0, r1;
  group_rows(R, r0, r1);
  float v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};      // dWmu[0..3], dWls[0..3], db1
  for (int rb = r0; rb < r1; rb += RPG) {
    float hh[RPG], dh[RPG], dm[RPG][4], dl[RPG][4];
#pragma unroll
    for (int t = 0; t < RPG; ++t) {
      const int r = min(rb + t, r1 - 1);
      const bool in = rb + t < r1;
      hh[t] = h1[(size_t)r * H + u];
      dh[t] = in ? dh1[(size_t)r * H + u] : 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int jj = min(j, A - 1);
        dm[t][j] = in ? dmu[(size_t)r * A + jj] : 0.0f;
        dl[t][j] = in ? dlsr[(size_t)r * A + jj] : 0.0f;
      }
    }
#pragma unroll
    for (int t = 0; t < RPG; ++t) {
      v[8] += dh[t];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] += dm[t][j] * hh[t];
        v[4 + j] += dl[t][j] * hh[t];
      }
    }
  }
  group_sum<9>(v, lds);
  if (threadIdx.x < CPB) {
    db1[u] = v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < A) {
        dwmu[(size_t)j * H + u] = v[j];
        dwls[(size_t)j * H + u] = v[4 + j];
      }
    }
  }
  if (blockIdx.x != 0 || threadIdx.x < 64) return;
  const int wv = (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;   // waves 1..3
  for (int j = 0; j < (wv == 3 ? 1 : A); ++j) {
    float part = 0.0f;
    for (int r = lane; r < R; r += 64) {
      if (wv == 1) part += dmu[(size_t)r * A + j];
      else if (wv == 2) part += dlsr[(size_t)r * A + j];
      else part += logp[r] + target_entropy;
    }
    const float sum = wave_sum(part);
    if (lane == 0) {
      if (wv == 1) dbmu[j] = sum;
      else if (wv == 2) dbls[j] = sum;
      else dlog_alpha[0] = -(sum / (float)R);
    }
  }
}

// m = dh0 (h0 > 0); dW0[u][k] = sum_r m x[r][k] (torch layout), db0[u] = sum_r m (x staged
// in LDS as above)
// dmu != nullptr: then the heads' column sums (actor_cols) in the same launch (its last step: the heads'
// and b1's column sums, d log_alpha; same rows, order and groups)
__global__ __launch_bounds__(256) void actor_bwd_in_kernel(
    const float* __restrict__ dh0, const float* __restrict__ h0, const float* __restrict__ x,
    int ldx, int K, int R, float* __restrict__ dw0, float* __restrict__ db0,
    const float* __restrict__ dmu, const float* __restrict__ dlsr, const float* __restrict__ h1,
    const float* __restrict__ dh1, const float* __restrict__ logp, float target_entropy, int A,
    float* __restrict__ dwmu, float* __restrict__ dwls, float* __restrict__ db1,
    float* __restrict__ dbmu, float* __restrict__ dbls, float* __restrict__ dlog_alpha) {
  __shared__ float lds[9][NRG][CPB];
  __shared__ float xl[kXR][kXK + 1];
  const int u = blockIdx.x * CPB + threadIdx.x % CPB;
  int r0, r1;
  group_rows(R, r0, r1);
  for (int q = threadIdx.x; q < R * K; q += blockDim.x) {
    const int r = q / K, k = q - r * K;
    xl[r][k] = x[(size_t)r * ldx + k];
  }
  float mm[RPG];
#pragma unroll
  for (int t = 0; t < RPG; ++t) {
    const int r = min(r0 + t, r1 - 1);
    const float h = h0[(size_t)r * H + u], d = dh0[(size_t)r * H + u];
    mm[t] = (r0 + t < r1 && h > 0.0f) ? d : 0.0f;
  }
  __syncthreads();
  for (int k0 = 0; k0 < K; k0 += 8) {
    float v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < RPG; ++t) {
      const int r = min(r0 + t, r1 - 1);
      v[8] += mm[t];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += mm[t] * xl[r][min(k0 + i, K - 1)];
    }
    group_sum<9>(v, lds);
    if (threadIdx.x < CPB) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (k0 + i < K) dw0[(size_t)u * K + k0 + i] = v[i];
      if (k0 == 0) db0[u] = v[8];
    }
  }
  if (dmu) actor_cols(dmu, dlsr, h1, dh1, logp, target_entropy, R, A, dwmu, dwls, db1, dbmu, dbls,
                      dlog_alpha, lds);
}

// C[b] = op(A[b]) op(B[b]) for the update's 256-wide products: op(A) is M x 256 (A row-major
// [M][256], or [256][M] transposed: TA), op(B) 256 x 256 (B row-major [256][256], or its
// transpose: TB), K = 256.  v_mfma_f32_16x16x4_f32 (f32 in, exact products, f32 accumulate):
// a workgroup of four waves takes one 16 x 16 tile of C, wave w the k range [64 w, 64 w + 64)
// in 16 steps (lane l: row l & 15 of op(A) / column l & 15 of op(B), k = 64 w + 16 (l >> 4)
// + step), then the four partial tiles are added in wave order through LDS -- M / 16 x 16
// tiles x batch workgroups, a short dependent chain per wave instead of rocBLAS's K loop.
#ifndef SF_GEMM_WAVES
#define SF_GEMM_WAVES 4
#endif
constexpr int kGW = SF_GEMM_WAVES;           // waves per tile (the K split)
constexpr int kGS = H / kGW / 4;             // MFMA steps per wave
template <bool TA, bool TB>
__global__ __launch_bounds__(64 * kGW) void gemm256_kernel(const float* __restrict__ A,
                                                           const float* __restrict__ Bm,
                                                           float* __restrict__ C, int M, long long sA,
                                                           long long sB, long long sC) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ float red[kGW][64][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col0 = blockIdx.x * 16, row0 = blockIdx.y * 16;
  const float* a = A + (size_t)blockIdx.z * sA;
  const float* b = Bm + (size_t)blockIdx.z * sB;
  const int i = lane & 15, g = lane >> 4;
  const int k0 = (H / kGW) * w + kGS * g;
  float av[kGS], bv[kGS];
#pragma unroll
  for (int m = 0; m < kGS; ++m) {
    av[m] = TA ? a[(size_t)(k0 + m) * M + row0 + i] : a[(size_t)(row0 + i) * H + k0 + m];
    bv[m] = TB ? b[(size_t)(col0 + i) * H + k0 + m] : b[(size_t)(k0 + m) * H + col0 + i];
  }
  f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int m = 0; m < kGS; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[m], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][lane][r] = acc[r];
  __syncthreads();
  if (w != 0) return;
  float* c = C + (size_t)blockIdx.z * sC;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = red[0][lane][r];
#pragma unroll
    for (int q = 1; q < kGW; ++q) v += red[q][lane][r];
    c[(size_t)(row0 + g * 4 + r) * H + col0 + i] = v;
  }
}

}  // namespace

#define SF_LAUNCH(kern, grid, block, ...)                                                    \
  do {                                                                                       \
    hipLaunchKernelGGL(kern, grid, block, 0, (hipStream_t)stream, __VA_ARGS__);              \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                         \
  } while (0)

extern "C" {

int32_t sf_gemm(int32_t ta, int32_t tb, const float* A, const float* B, float* C, int32_t M, int32_t batch,
                long long sA, long long sB, long long sC, void* stream) {
  if (!A || !B || !C || M < 16 || (M % 16) != 0 || batch < 1) return -1;
  const dim3 grid(H / 16, M / 16, batch);
  const dim3 blk(64 * kGW);
  if (ta && tb) SF_LAUNCH((gemm256_kernel<true, true>), grid, blk, A, B, C, M, sA, sB, sC);
  if (ta) SF_LAUNCH((gemm256_kernel<true, false>), grid, blk, A, B, C, M, sA, sB, sC);
  if (tb) SF_LAUNCH((gemm256_kernel<false, true>), grid, blk, A, B, C, M, sA, sB, sC);
  SF_LAUNCH((gemm256_kernel<false, false>), grid, blk, A, B, C, M, sA, sB, sC);
}

int32_t sf_in_layer(const float* xa, const float* xa_hi, int32_t split, int32_t lda, int32_t Ka,
                    const float* xb, int32_t ldb, int32_t Kb, int32_t R, int32_t nC, const float* w,
                    int32_t w_ku, const float* b, float* out, void* stream) {
  if (!xa || !w || !b || !out || R < 1 || nC < 1 || nC > 2 || Ka < 1 || Kb < 0 || (Kb && !xb) ||
      (!w_ku && nC != 1))
    return -1;
  if (!xa_hi) { xa_hi = xa; split = R; }
  SF_LAUNCH(in_layer_kernel, dim3(R, nC), dim3(H), xa, xa_hi, split, lda, Ka, xb, ldb, Kb, R, nC, w,
            w_ku, b, out);
}

int32_t sf_actor_head(const float* p1, const float* b1, const float* wmu, const float* bmu,
                      const float* wls, const float* bls, const float* eps, int32_t R, int32_t A,
                      float* h1, float* mu, float* lsr, float* a_out, float* logp, int32_t RT,
                      const float* xt, int32_t ldxt, int32_t Kxt, const float* tw0, const float* tb0,
                      float* g0t, void* stream) {
  if (!p1 || !b1 || !wmu || !bmu || !wls || !bls || !eps || !h1 || !mu || !lsr || !a_out || !logp ||
      R < 1 || A < 1 || A > 4)
    return -1;
  if (g0t && (!xt || !tw0 || !tb0 || RT < 1 || RT > R || Kxt < 1 || ldxt < Kxt)) return -1;
  SF_LAUNCH(actor_head_kernel, dim3((R + 3) / 4), dim3(256), p1, b1, wmu, bmu, wls, bls, eps, R, A,
            h1, mu, lsr, a_out, logp, RT, xt, ldxt, Kxt, tw0, tb0, g0t);
}

int32_t sf_in_layer_pair(const float* xa, const float* xa_hi, int32_t split, int32_t lda, int32_t Ka,
                         int32_t R1, const float* w1, const float* b1, float* out1, const float* ya,
                         int32_t ldya, int32_t Kya, const float* yb, int32_t ldyb, int32_t Kyb, int32_t R2,
                         const float* w2, const float* b2, float* out2, void* stream) {
  if (!xa || !xa_hi || !w1 || !b1 || !out1 || !ya || !w2 || !b2 || !out2 || R1 < 1 || R2 < 1 ||
      Ka < 1 || Kya < 1 || Kyb < 0 || (Kyb && !yb) || split < 0 || split > R1)
    return -1;
  const int R = R1 > R2 ? R1 : R2;
  SF_LAUNCH(in_layer_pair_kernel, dim3(R, 3), dim3(H), xa, xa_hi, split, lda, Ka, R1, w1, b1, out1,
            ya, ldya, Kya, yb, ldyb, Kyb, R2, w2, b2, out2);
}

int32_t sf_noise_sample(unsigned long long* launch, unsigned long long seed, float* u, int32_t nu,
                        float* e1, int32_t n1, float* e2, int32_t n2, const float* buf, long long cap,
                        int32_t W, const long long* size, float* rows, float* step, void* stream) {
  if (!launch || nu < 1 || nu > 1024 || n1 < 0 || n2 < 0 || !u || (n1 && !e1) || (n2 && !e2) || !buf ||
      cap < 1 || W < 1 || !size || !rows || !step)
    return -1;
  SF_LAUNCH(noise_sample_kernel, dim3(1), dim3(1024), launch, seed, u, nu, e1, n1, e2, n2, buf, cap, W, size,
            rows, step);
}

int32_t sf_noise(unsigned long long* launch, unsigned long long seed, float* u, int32_t nu, float* e1,
                 int32_t n1, float* e2, int32_t n2, void* stream) {
  if (!launch || nu < 0 || n1 < 0 || n2 < 0 || (nu && !u) || (n1 && !e1) || (n2 && !e2)) return -1;
  SF_LAUNCH(noise_kernel, dim3(1), dim3(1024), launch, seed, u, nu, e1, n1, e2, n2);
}

int32_t sf_critic_head(const float* p1, const float* b1, const float* w2, const float* b2, int32_t B,
                       int32_t mode, const float* rows, int32_t W, int32_t col_r, int32_t col_d,
                       float gamma, const float* log_alpha, const float* logp, float* y, float* g1,
                       float* q_out, float* dq, float* dlogp, float* lossp, float* dg1, void* stream) {
  if (!p1 || !b1 || !w2 || !b2 || !log_alpha || !q_out || B < 1 || mode < 0 || mode > 2) return -1;
  if (mode == HEAD_TARGET && (!rows || !logp || !y || col_r < 0 || col_r >= W || col_d < 0 || col_d >= W))
    return -1;
  if (mode == HEAD_CRITIC && (!y || !g1 || !dq || !lossp)) return -1;
  if (mode == HEAD_ACTOR_LOSS && (!logp || !(g1 || dg1) || !dq || !dlogp || !lossp)) return -1;
  SF_LAUNCH(critic_head_kernel, dim3((B + 3) / 4), dim3(256), p1, b1, w2, b2, B, mode, rows, W, col_r,
            col_d, gamma, log_alpha, logp, y, g1, q_out, dq, dlogp, lossp, dg1);
}

int32_t sf_critic_bwd_in(const float* dg0, const float* g0, const float* xa, int32_t lda, int32_t Ka,
                         const float* xb, int32_t ldb, int32_t Kb, int32_t B, float* dw0, float* db0,
                         const float* g1, const float* dq, const float* w2, float* dw2, float* db1,
                         float* db2, void* stream) {
  if (g1 && (!dq || !w2 || !dw2 || !db1 || !db2)) return -1;
  if (!dg0 || !g0 || !xa || !dw0 || !db0 || B < 1 || Ka < 1 || Kb < 0 || (Kb && !xb)) return -1;
  if (B > kXR || Ka + Kb > kXK || B > NRG * RPG) return -1;
  SF_LAUNCH(critic_bwd_in_kernel, dim3(H / CPB, 2), dim3(256), dg0, g0, xa, lda, Ka, xb, ldb, Kb, B, dw0, db0,
            g1, dq, w2, dw2, db1, db2);
}

int32_t sf_actor_bwd_head(const float* ga, const float* gl, const float* mu, const float* lsr,
                          const float* eps, const float* a_out, const float* h1, const float* wmu,
                          const float* wls, int32_t R, int32_t A, float* dmu, float* dlsr, float* dh1,
                          const float* dg0, const float* g0, const float* w0, int32_t K, int32_t Ka,
                          void* stream) {
  if (!gl || !mu || !lsr || !eps || !a_out || !h1 || !wmu || !wls || !dmu || !dlsr || !dh1 ||
      R < 1 || A < 1 || A > 4)
    return -1;
  if (!ga && (!dg0 || !g0 || !w0 || Ka < 0 || Ka + A > K)) return -1;
  SF_LAUNCH(actor_bwd_head_kernel, dim3((R + 3) / 4), dim3(256), ga, gl, mu, lsr, eps, a_out, h1, wmu,
            wls, R, A, dmu, dlsr, dh1, dg0, g0, w0, K, Ka);
}

int32_t sf_td_critic_head(const float* p1, const float* tb1, const float* tw2, const float* tb2,
                          const float* b1, const float* w2, const float* b2, int32_t B, const float* rows,
                          int32_t W, int32_t col_r, int32_t col_d, float gamma, const float* log_alpha,
                          const float* logp, float* y, float* g1, float* q_out, float* dq, float* lossp,
                          float* dg1, void* stream) {
  if (!p1 || !tb1 || !tw2 || !tb2 || !b1 || !w2 || !b2 || !rows || !log_alpha || !logp || !y || !g1 ||
      !q_out || !dq || !lossp || B < 1 || col_r < 0 || col_r >= W || col_d < 0 || col_d >= W)
    return -1;
  SF_LAUNCH(td_critic_head_kernel, dim3((B + 3) / 4), dim3(256), p1, tb1, tw2, tb2, b1, w2, b2, B, rows,
            W, col_r, col_d, gamma, log_alpha, logp, y, g1, q_out, dq, lossp, dg1);
}

int32_t sf_actor_bwd_in(const float* dh0, const float* h0, const float* x, int32_t ldx, int32_t K,
                        int32_t R, float* dw0, float* db0, const float* dmu, const float* dlsr,
                        const float* h1, const float* dh1, const float* logp, float target_entropy,
                        int32_t A, float* dwmu, float* dwls, float* db1, float* dbmu, float* dbls,
                        float* dlog_alpha, void* stream) {
  if (dmu && (!dlsr || !h1 || !dh1 || !logp || !dwmu || !dwls || !db1 || !dbmu || !dbls || !dlog_alpha ||
              A < 1 || A > 4))
    return -1;
  if (!dh0 || !h0 || !x || !dw0 || !db0 || R < 1 || K < 1) return -1;
  if (R > kXR || K > kXK || R > NRG * RPG) return -1;
  SF_LAUNCH(actor_bwd_in_kernel, dim3(H / CPB), dim3(256), dh0, h0, x, ldx, K, R, dw0, db0, dmu, dlsr, h1,
            dh1, logp, target_entropy, A, dwmu, dwls, db1, dbmu, dbls, dlog_alpha);
}

}  // extern "C"
