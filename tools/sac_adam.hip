// Learner kernels of the C5 bench (tools/sac_torch.py).
//
// Adam step: every parameter tensor of one or more
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

struct polyak_targets {
  float* t[SAC_ADAM_MAX_TENSORS];
};

// tgt (optional): SB3's polyak_update of a target copy of each parameter, fused behind its Adam
// step -- target = target (1 - tau) + tau * p_new (FusedSAC: the critic's parameters change only
// in this step of an update, so the target update may follow it directly)
__global__ __launch_bounds__(BLOCK) void adam_kernel(sac_adam_table T, const float* __restrict__ step,
                                                      float lr, float b1, float b2, float eps,
                                                      polyak_targets tgt, float tau, int has_tgt) {
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
  const float pn = T.p[i][k] - (lr / bc1) * m / denom;
  T.p[i][k] = pn;
  if (has_tgt) {
    const float t0 = tgt.t[i][k] * (1.0f - tau);
    tgt.t[i][k] = t0 + tau * pn;
  }
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
  polyak_targets none{};
  hipLaunchKernelGGL(adam_kernel, dim3(T->start[T->n]), dim3(BLOCK), 0, (hipStream_t)stream, *T,
                     step, lr, b1, b2, eps, none, 0.0f, 0);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// the Adam step above with each parameter's target copy polyak-updated behind it (tgt[i] has
// T->numel[i] elements)
extern "C" int32_t sac_adam_step_polyak(const sac_adam_table* T, const float* step, float lr, float b1,
                                        float b2, float eps, float* const* tgt, float tau, void* stream) {
  if (!T || !step || !tgt || T->n < 1 || T->n > SAC_ADAM_MAX_TENSORS) return -1;
  polyak_targets pt{};
  for (int i = 0; i < T->n; ++i) {
    if (!T->p[i] || !T->g[i] || !T->m[i] || !T->v[i] || !tgt[i] || T->numel[i] <= 0) return -1;
    if (T->start[i + 1] - T->start[i] != (int32_t)((T->numel[i] + BLOCK - 1) / BLOCK)) return -1;
    pt.t[i] = tgt[i];
  }
  if (T->start[0] != 0) return -1;
  hipLaunchKernelGGL(adam_kernel, dim3(T->start[T->n]), dim3(BLOCK), 0, (hipStream_t)stream, *T,
                     step, lr, b1, b2, eps, pt, tau, 1);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------------------
// Replay insert for the C5 learner: the E transitions of one vector step written as packed
// rows [obs | act | reward | next_obs | terminated] at ring positions (pos + e) % cap, in ONE
// launch (the torch form is ~12 kernels: arange/add/remainder for the indices, the
// terminated|truncated mask, torch.where for next_obs, casts, cat, index_copy, the pos/size
// updates).  next_obs is the terminal observation (final_obs) for envs that ended this step
// (terminated or truncated), as SB3's VecEnv hands it over; `terminated` alone is the done
// flag (SB3 handle_timeout_termination).  pos / size (int64, device) are read by every
// workgroup at its start and advanced by the last workgroup to finish (ticket counter), so
// the launch is graph-capturable.  Pure copies and exact casts: bit-identical to the torch form.
namespace {

__global__ __launch_bounds__(256) void replay_insert_kernel(
    float* __restrict__ buf, long long cap, int O, int A, const float* obs,
    const double* __restrict__ act, const float* __restrict__ rew, const uint8_t* __restrict__ term,
    const uint8_t* __restrict__ trunc, const float* __restrict__ next_obs,
    const float* __restrict__ final_obs, int E, long long* pos, long long* size, unsigned* ticket,
    float* obs_out) {
  const int W = 2 * O + A + 2;
  const long long p0 = __atomic_load_n(pos, __ATOMIC_RELAXED);
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (long long)E * W) {
    const int e = (int)(i / W), c = (int)(i - (long long)e * W);
    float v;
    if (c < O) {
      // obs_out (the loop's observation buffer) may be obs itself, so neither pointer is
      // __restrict__: the compiler may not move this load after the store below (ADVICE
      // r05).  This thread alone reads and writes element (e, c).
      v = obs[(size_t)e * O + c];
      if (obs_out) obs_out[(size_t)e * O + c] = next_obs[(size_t)e * O + c];
    } else if (c < O + A) {
      v = (float)act[(size_t)e * A + (c - O)];
    } else if (c == O + A) {
      v = rew[e];
    } else if (c < 2 * O + A + 1) {
      const int k = c - (O + A + 1);
      v = (term[e] | trunc[e]) ? final_obs[(size_t)e * O + k] : next_obs[(size_t)e * O + k];
    } else {
      v = (float)term[e];
    }
    buf[(size_t)((p0 + e) % cap) * W + c] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned t = atomicAdd(ticket, 1u);
    if (t == gridDim.x - 1) {                     // every workgroup has read pos
      const long long s = __atomic_load_n(size, __ATOMIC_RELAXED) + E;
      atomicExch(reinterpret_cast<unsigned long long*>(pos), (unsigned long long)((p0 + E) % cap));
      atomicExch(reinterpret_cast<unsigned long long*>(size), (unsigned long long)(s < cap ? s : cap));
      atomicExch(ticket, 0u);
    }
  }
}

}  // namespace

extern "C" int32_t sac_replay_insert(float* buf, long long cap, int32_t obs_dim, int32_t act_dim,
                                     const float* obs, const double* act, const float* rew,
                                     const uint8_t* term, const uint8_t* trunc,
                                     const float* next_obs, const float* final_obs, int32_t E,
                                     long long* pos, long long* size, unsigned* ticket,
                                     void* stream) {
  if (!buf || cap < 1 || obs_dim < 1 || act_dim < 1 || E < 1 || E > cap || !obs || !act || !rew ||
      !term || !trunc || !next_obs || !final_obs || !pos || !size || !ticket)
    return -1;
  const long long n = (long long)E * (2 * obs_dim + act_dim + 2);
  const int grid = (int)((n + 255) / 256);
  hipLaunchKernelGGL(replay_insert_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, buf, cap,
                     obs_dim, act_dim, obs, act, rew, term, trunc, next_obs, final_obs, E, pos, size,
                     ticket, nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// the insert above that also copies the post-step observations into obs_out (RLLoop's obs
// buffer, which may be `obs` itself) -- the loop's separate copy launch folded in
extern "C" int32_t sac_replay_insert_obs(float* buf, long long cap, int32_t obs_dim, int32_t act_dim,
                                         const float* obs, const double* act, const float* rew,
                                         const uint8_t* term, const uint8_t* trunc,
                                         const float* next_obs, const float* final_obs, int32_t E,
                                         long long* pos, long long* size, unsigned* ticket,
                                         float* obs_out, void* stream) {
  if (!buf || cap < 1 || obs_dim < 1 || act_dim < 1 || E < 1 || E > cap || !obs || !act || !rew ||
      !term || !trunc || !next_obs || !final_obs || !pos || !size || !ticket || !obs_out)
    return -1;
  const long long n = (long long)E * (2 * obs_dim + act_dim + 2);
  const int grid = (int)((n + 255) / 256);
  hipLaunchKernelGGL(replay_insert_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, buf, cap,
                     obs_dim, act_dim, obs, act, rew, term, trunc, next_obs, final_obs, E, pos, size,
                     ticket, obs_out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------------------
// Replay sample for the C5 learner: rows buf[min((int64)(u_b * (float)size), cap - 1)] for the
// batch's uniforms u (torch.rand, fp32) gathered into a contiguous [B, W] tile in ONE launch
// (the torch form: a size cast, mul, long cast, clamp and an index gather).  The index
// arithmetic is the torch form's, operation for operation (fp32 product, truncation toward
// zero, clamp), so the rows drawn are the same.
namespace {

__global__ __launch_bounds__(256) void replay_sample_kernel(const float* __restrict__ buf, long long cap,
                                                           int W, const float* __restrict__ u, int B,
                                                           const long long* __restrict__ size,
                                                           float* __restrict__ out,
                                                           float* __restrict__ tick) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tick && i == 0) tick[0] += 1.0f;     // HipAdam.tick (t.add_(1.0)) folded in: no reader here
  if (i >= (long long)B * W) return;
  const int b = (int)(i / W), c = (int)(i - (long long)b * W);
  long long idx = (long long)(u[b] * (float)size[0]);
  if (idx > cap - 1) idx = cap - 1;
  out[i] = buf[(size_t)idx * W + c];
}

}  // namespace

extern "C" int32_t sac_replay_sample(const float* buf, long long cap, int32_t row_width,
                                     const float* u, int32_t batch, const long long* size,
                                     float* out, void* stream) {
  if (!buf || cap < 1 || row_width < 1 || !u || batch < 1 || !size || !out) return -1;
  const long long n = (long long)batch * row_width;
  hipLaunchKernelGGL(replay_sample_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, buf, cap, row_width, u, batch, size, out, nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// the sample above with the optimizers' device step count advanced in the same launch
// (FusedSAC: one launch less per update; the count is read only by the Adam launches after it)
extern "C" int32_t sac_replay_sample_tick(const float* buf, long long cap, int32_t row_width,
                                          const float* u, int32_t batch, const long long* size,
                                          float* out, float* step, void* stream) {
  if (!buf || cap < 1 || row_width < 1 || !u || batch < 1 || !size || !out || !step) return -1;
  const long long n = (long long)batch * row_width;
  hipLaunchKernelGGL(replay_sample_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, buf, cap, row_width, u, batch, size, out, step);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------------------
// SAC TD target for the C5 learner: y = r + gamma * (1 - d) * (min(q_t1, q_t2) - alpha * logp')
// in ONE launch (the torch form is six: amin, mul, sub, rsub, mul, mul, add), operation for
// operation in fp32 without contraction (this file builds with -ffp-contract=off), so y is
// bit-identical.  r and d are columns of the sampled rows [B, W] (col_r, col_d).
namespace {

__global__ __launch_bounds__(256) void td_target_kernel(const float* __restrict__ q2, const float* __restrict__ logp2,
                                                       const float* __restrict__ alpha,
                                                       const float* __restrict__ rows, int W, int col_r,
                                                       int col_d, float gamma, int B, float* __restrict__ y) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float q = fminf(q2[b], q2[B + b]);
  const float qt = q - alpha[0] * logp2[b];
  const float d = rows[(size_t)b * W + col_d];
  const float r = rows[(size_t)b * W + col_r];
  y[b] = r + (gamma * (1.0f - d)) * qt;
}

}  // namespace

extern "C" int32_t sac_td_target(const float* q2, const float* logp2, const float* alpha,
                                 const float* rows, int32_t W, int32_t col_r, int32_t col_d,
                                 float gamma, int32_t B, float* y, void* stream) {
  if (!q2 || !logp2 || !alpha || !rows || !y || B < 1 || W < 1 || col_r < 0 || col_r >= W ||
      col_d < 0 || col_d >= W)
    return -1;
  hipLaunchKernelGGL(td_target_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, q2,
                     logp2, alpha, rows, W, col_r, col_d, gamma, B, y);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------------------
// Twin-critic MSE for the C5 learner: loss = sum_c mean_b (q[c, b] - y[b])^2 and the saved
// difference q - y in ONE launch (one workgroup; B <= 1024), and its backward
// dq = (g / B) * (2 (q - y)) in one more -- the operation order of torch's autograd for
// (q - y).pow(2).mean(-1).sum() (MeanBackward divides the incoming gradient by B, PowBackward
// multiplies by 2 (q - y)), so the gradient is bit-identical; the loss value itself comes
// from a different reduction order (it is only reported).
namespace {

__global__ __launch_bounds__(1024) void twin_mse_fwd_kernel(const float* __restrict__ q,
                                                            const float* __restrict__ y, int B,
                                                            float* __restrict__ diff, float* __restrict__ loss) {
  __shared__ float part[1024 / 64];
  float acc = 0.0f;
  for (int i = threadIdx.x; i < 2 * B; i += blockDim.x) {
    const float d = q[i] - y[i % B];
    diff[i] = d;
    acc += d * d / (float)B;
  }
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
    loss[0] = s;
  }
}

__global__ __launch_bounds__(256) void twin_mse_bwd_kernel(const float* __restrict__ diff,
                                                           const float* __restrict__ g, int B,
                                                           float* __restrict__ dq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * B) return;
  dq[i] = (g[0] / (float)B) * (2.0f * diff[i]);
}

}  // namespace

extern "C" int32_t sac_twin_mse_fwd(const float* q, const float* y, int32_t B, float* diff,
                                    float* loss, void* stream) {
  if (!q || !y || !diff || !loss || B < 1) return -1;
  hipLaunchKernelGGL(twin_mse_fwd_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, q, y, B,
                     diff, loss);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int32_t sac_twin_mse_bwd(const float* diff, const float* g, int32_t B, float* dq,
                                    void* stream) {
  if (!diff || !g || !dq || B < 1) return -1;
  hipLaunchKernelGGL(twin_mse_bwd_kernel, dim3((2 * B + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, diff, g, B, dq);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------------------
// SAC actor loss for the C5 learner: loss = mean_b(alpha * logp[b] - min(q[0, b], q[1, b])) in
// one launch (one workgroup; B <= 1024), backward in one more: dlogp = (g / B) * alpha and
// dq[c, b] = -(g / B) on the smaller critic (split evenly on a tie), autograd's operation
// order for (alpha * logp - q.amin(0)).mean() (MeanBackward's g / B, MulBackward's * alpha,
// SubBackward's negation, AminBackward's even split).  The loss value comes from a different
// reduction order (reported only).
namespace {

__global__ __launch_bounds__(1024) void actor_loss_fwd_kernel(const float* __restrict__ q,
                                                              const float* __restrict__ logp,
                                                              const float* __restrict__ alpha, int B,
                                                              float* __restrict__ loss) {
  __shared__ float part[1024 / 64];
  float acc = 0.0f;
  const float al = alpha[0];
  for (int b = threadIdx.x; b < B; b += blockDim.x) acc += (al * logp[b] - fminf(q[b], q[B + b])) / (float)B;
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
    loss[0] = s;
  }
}

__global__ __launch_bounds__(256) void actor_loss_bwd_kernel(const float* __restrict__ q,
                                                             const float* __restrict__ alpha,
                                                             const float* __restrict__ g, int B,
                                                             float* __restrict__ dq, float* __restrict__ dlogp) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float gb = g[0] / (float)B;
  dlogp[b] = gb * alpha[0];
  const float q0 = q[b], q1 = q[B + b], mn = fminf(q0, q1);
  const float ng = -gb;
  if (q0 == q1) {
    dq[b] = ng / 2.0f;
    dq[B + b] = ng / 2.0f;
  } else {
    dq[b] = q0 == mn ? ng : 0.0f;
    dq[B + b] = q1 == mn ? ng : 0.0f;
  }
}

}  // namespace

extern "C" int32_t sac_actor_loss_fwd(const float* q, const float* logp, const float* alpha, int32_t B,
                                      float* loss, void* stream) {
  if (!q || !logp || !alpha || !loss || B < 1) return -1;
  hipLaunchKernelGGL(actor_loss_fwd_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, q, logp,
                     alpha, B, loss);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int32_t sac_actor_loss_bwd(const float* q, const float* alpha, const float* g, int32_t B,
                                      float* dq, float* dlogp, void* stream) {
  if (!q || !alpha || !g || !dq || !dlogp || B < 1) return -1;
  hipLaunchKernelGGL(actor_loss_bwd_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     q, alpha, g, B, dq, dlogp);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------------------
// SB3's squashed diagonal Gaussian for the C5 learner's actor pass, one launch forward and
// one backward (the torch form is ~13 elementwise kernels forward and as many backward):
//   ls = clamp(ls_raw, -20, 2); std = exp(ls); u = mu + std * eps; a = tanh(u);
//   logp = sum_j [-((u - mu) / std)^2 / 2 - ls - log(2 pi) / 2] - sum_j log(1 - a^2 + 1e-6)
// backward from (ga, gl): with z = (u - mu) / std,
//   g_u = ga (1 - a^2) + gl (-z / std + 2a (1 - a^2) / (1 - a^2 + 1e-6))
//   g_mu = g_u + gl z / std;  g_std = g_u eps + gl z^2 / std;  g_ls = g_std std - gl,
//   passed to ls_raw inside the clamp's closed range (torch's clamp backward).
// One thread per row (A <= 4).  Within fp32 rounding of torch's autograd (different
// association), checked by tests/test_gpu_sac_adam.py.
namespace {

__global__ __launch_bounds__(256) void sq_gauss_fwd_kernel(const float* __restrict__ mu, const float* __restrict__ lsr,
                                                          const float* __restrict__ eps, int N, int A,
                                                          float* __restrict__ a_out, float* __restrict__ logp) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  float s1 = 0.0f, s2 = 0.0f;
  for (int j = 0; j < A; ++j) {
    const int i = r * A + j;
    const float ls = fminf(fmaxf(lsr[i], -20.0f), 2.0f);
    const float sd = expf(ls);
    const float u = mu[i] + sd * eps[i];
    const float a = tanhf(u);
    a_out[i] = a;
    const float z = (u - mu[i]) / sd;
    s1 += -0.5f * (z * z) - ls - 0.91893853320467274f;
    s2 += logf(1.0f - a * a + 1e-6f);
  }
  logp[r] = s1 - s2;
}

__global__ __launch_bounds__(256) void sq_gauss_bwd_kernel(const float* __restrict__ mu, const float* __restrict__ lsr,
                                                          const float* __restrict__ eps, const float* __restrict__ a_out,
                                                          const float* __restrict__ ga, const float* __restrict__ gl,
                                                          int N, int A, float* __restrict__ gmu,
                                                          float* __restrict__ glsr) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const float g = gl ? gl[r] : 0.0f;
  for (int j = 0; j < A; ++j) {
    const int i = r * A + j;
    const float x = lsr[i];
    const float ls = fminf(fmaxf(x, -20.0f), 2.0f);
    const float sd = expf(ls);
    const float u = mu[i] + sd * eps[i];
    const float z = (u - mu[i]) / sd;
    const float a = a_out[i];
    const float da = 1.0f - a * a;
    const float gu = (ga ? ga[i] : 0.0f) * da + g * (-z / sd + (2.0f * a / (da + 1e-6f)) * da);
    gmu[i] = gu + g * z / sd;
    const float gsd = gu * eps[i] + g * (z * z) / sd;
    const float gls = gsd * sd - g;
    glsr[i] = (x >= -20.0f && x <= 2.0f) ? gls : 0.0f;
  }
}

}  // namespace

extern "C" int32_t sac_sq_gauss_fwd(const float* mu, const float* lsr, const float* eps, int32_t N,
                                    int32_t A, float* a_out, float* logp, void* stream) {
  if (!mu || !lsr || !eps || !a_out || !logp || N < 1 || A < 1 || A > 4) return -1;
  hipLaunchKernelGGL(sq_gauss_fwd_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     mu, lsr, eps, N, A, a_out, logp);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int32_t sac_sq_gauss_bwd(const float* mu, const float* lsr, const float* eps,
                                    const float* a_out, const float* ga, const float* gl, int32_t N,
                                    int32_t A, float* gmu, float* glsr, void* stream) {
  if (!mu || !lsr || !eps || !a_out || !gmu || !glsr || N < 1 || A < 1 || A > 4) return -1;
  hipLaunchKernelGGL(sq_gauss_bwd_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     mu, lsr, eps, a_out, ga, gl, N, A, gmu, glsr);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
