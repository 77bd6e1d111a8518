// Host cost of the per-step stream bookkeeping of the multi-GPU learner-row gather, with a
// ~28 us kernel standing in for a C4 8-GPU shard's step (the regime where the host, not the
// GPU, bounds a sharded step: profiles/r04/comm/shard_overhead.txt).  One GPU, a one-rank
// RCCL communicator (the same enqueue path as on the node).  Diagnostic only.
//
//   hipcc -O2 --offload-arch=gfx950 -o tools/probe/hostapi_probe tools/probe/hostapi_probe.cpp -ldl
//   tools/probe/hostapi_probe [spin_us]
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef struct ncclComm* ncclComm_t;
typedef struct { char internal[128]; } ncclUniqueId;
static int (*p_get_id)(ncclUniqueId*);
static int (*p_init)(ncclComm_t*, int, ncclUniqueId, int);
static int (*p_ag)(const void*, void*, size_t, int, ncclComm_t, hipStream_t);

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void spin(long long cycles, float* rows, int n) {
  // bounded: every wave leaves after `cycles` of the 100 MHz constant clock
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {}
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) rows[i] += 1.0f;
}

// the spin kernel whose last workgroup publishes "step seq done" (a release store at system
// scope after every workgroup's rows are out): the side stream waits for that value instead of
// an event recorded behind the kernel
__global__ void spin_flag(long long cycles, float* rows, int n, unsigned* count, uint64_t* flag, uint64_t seq) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {}
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) rows[i] += 1.0f;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(count, 1u);
    if (prev == gridDim.x - 1) {
      __threadfence();
      *count = 0u;
      __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const double spin_us = argc > 1 ? std::atof(argv[1]) : 28.0;
  void* h = dlopen("librccl.so.1", RTLD_NOW);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
  if (!h) { std::printf("no rccl\n"); return 1; }
  p_get_id = (decltype(p_get_id))dlsym(h, "ncclGetUniqueId");
  p_init = (decltype(p_init))dlsym(h, "ncclCommInitRank");
  p_ag = (decltype(p_ag))dlsym(h, "ncclAllGather");
  CK(hipSetDevice(0));
  ncclUniqueId id;
  p_get_id(&id);
  ncclComm_t nc;
  if (p_init(&nc, 1, id, 0) != 0) { std::printf("ncclCommInitRank failed\n"); return 1; }
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  const int R = 16;
  const size_t n = 512 * 43;                  // a 512-env shard's learner rows (fp32)
  float *rows, *gath;
  CK(hipMalloc(&rows, R * n * 4));
  CK(hipMalloc(&gath, R * n * 4));
  uint64_t* flag;
  CK(hipMalloc(&flag, 64));
  CK(hipMemset(flag, 0, 64));
  unsigned* count;
  CK(hipMalloc(&count, 64));
  CK(hipMemset(count, 0, 64));
  uint64_t kseq = 0;
  hipEvent_t ea[R], eb[R];
  for (int i = 0; i < R; ++i) {
    CK(hipEventCreateWithFlags(&ea[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eb[i], hipEventDisableTiming));
  }
  const long long cyc = (long long)(spin_us * 100.0);    // wall_clock64: 100 MHz
  const int T = 2000;
  struct Acc { double launch = 0, rec = 0, wait = 0, coll = 0, rec2 = 0, rwait = 0; };
  hipStream_t Bdef = B;
  auto run = [&](const char* name, int variant) {
    Acc a;
    uint64_t seq = 0;
    int last_fence = -1000000;          // step of the newest recorded gather fence
    int waited = -1000000;              // gathers <= waited are known done on A
    std::vector<int> fence_step(R, -1);
    for (int warm = 0; warm < 2; ++warm) {
      CK(hipDeviceSynchronize());
      a = Acc();
      const double w0 = now_us();
      for (int t = 0; t < T; ++t) {
        const int s = t % R;
        double t0 = now_us();
        // reverse dependency: rows[s] was read by the gather of step t - R (or t - 2 at R = 2)
        if (variant == 1) {
          if (t >= 2) CK(hipStreamWaitEvent(A, eb[t % 2], 0));
        } else if (variant >= 2 && variant <= 8) {
          if (t - R > waited) {
            // the oldest fence that covers step t - R
            int best = -1;
            for (int k = 0; k < R; ++k)
              if (fence_step[k] >= t - R && (best < 0 || fence_step[k] < fence_step[best])) best = k;
            if (best >= 0) { CK(hipStreamWaitEvent(A, eb[best], 0)); waited = fence_step[best]; }
          }
        }
        double t1 = now_us();
        if (variant == 8)
          hipLaunchKernelGGL(spin_flag, dim3(64), dim3(64), 0, A, cyc, rows + (size_t)s * n, (int)n, count, flag, ++kseq);
        else
          hipLaunchKernelGGL(spin, dim3(64), dim3(64), 0, A, cyc, rows + (size_t)(variant == 1 ? t % 2 : s) * n, (int)n);
        double t2 = now_us();
        double t3 = t2, t4 = t2, t5 = t2;
        if (variant == 0) {
          // launch only
        } else if (variant == 5) {
          // the gather on the compute stream itself (no cross-stream sync; serialised)
          p_ag(rows + (size_t)s * n, gath + (size_t)s * n, n, 7, nc, A);
          t4 = now_us(); t5 = t4; t3 = t2;
        } else {
          if (variant == 8) {
            t3 = now_us();
            CK(hipStreamWaitValue64(B, flag, kseq, hipStreamWaitValueGte, ~0ull));
          } else if (variant == 4) {
            ++seq;
            CK(hipStreamWriteValue64(A, flag, seq, 0));
            t3 = now_us();
            CK(hipStreamWaitValue64(B, flag, seq, hipStreamWaitValueGte, ~0ull));
          } else {
            const int es = variant == 1 ? t % 2 : s;
            CK(hipEventRecord(ea[es], A));
            t3 = now_us();
            CK(hipStreamWaitEvent(B, ea[es], 0));
          }
          t4 = now_us();
          p_ag(rows + (size_t)(variant == 1 ? t % 2 : s) * n, gath + (size_t)(variant == 1 ? t % 2 : s) * n, n, 7, nc, B);
          t5 = now_us();
          if (variant == 1) {
            CK(hipEventRecord(eb[t % 2], B));
          } else if (t % (R / 2) == 0) {        // a fence every R/2 gathers
            const int slot = (t / (R / 2)) % R;
            CK(hipEventRecord(eb[slot], B));
            fence_step[slot] = t;
            last_fence = t;
          }
        }
        double t6 = now_us();
        a.rwait += t1 - t0; a.launch += t2 - t1; a.rec += t3 - t2; a.wait += t4 - t3;
        a.coll += t5 - t4; a.rec2 += t6 - t5;
      }
      CK(hipDeviceSynchronize());
      const double wall = (now_us() - w0) / T;
      if (warm == 1) {
        const double host = (a.rwait + a.launch + a.rec + a.wait + a.coll + a.rec2) / T;
        std::printf("%-58s wall/step %6.1f us  host/step %6.1f us | rwait %5.2f launch %5.2f "
                    "fwd-rec %5.2f fwd-wait %5.2f gather %5.2f fence %5.2f\n", name, wall, host,
                    a.rwait / T, a.launch / T, a.rec / T, a.wait / T, a.coll / T, a.rec2 / T);
      }
    }
    (void)last_fence;
  };
  std::printf("spin kernel %.1f us, %d steps per variant, R = %d row slots\n", spin_us, T, R);
  run("launch only", 0);
  run("events: fwd record+wait, reverse wait every step (R=2)", 1);
  run("events: fwd record+wait, fence + reverse wait per R/2", 2);
  run("writeValue/waitValue fwd, fence + reverse wait per R/2", 4);
  run("gather on the compute stream (serialised)", 5);
  run("kernel-written flag + waitValue, fence per R/2", 8);
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  std::printf("stream priority range: least %d greatest %d\n", lo, hi);
  hipStream_t Bh, Bl;
  CK(hipStreamCreateWithPriority(&Bh, hipStreamNonBlocking, hi));
  CK(hipStreamCreateWithPriority(&Bl, hipStreamNonBlocking, lo));
  B = Bh;
  run("[B high priority] kernel-written flag + waitValue, fence per R/2", 8);
  run("[B high priority] events, fence per R/2", 2);
  run("[B high priority] writeValue/waitValue, fence per R/2", 4);
  run("[B high priority] events, reverse wait every step (R=2)", 1);
  B = Bl;
  run("[B low priority] events, fence per R/2", 2);
  // more plain streams: shift which hardware queue the next stream lands on
  for (int k = 0; k < 3; ++k) {
    hipStream_t x;
    CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, x, 10LL, rows, 0);
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, B, 10LL, rows, 0);
    CK(hipDeviceSynchronize());
    char nm[96];
    std::snprintf(nm, sizeof(nm), "[new B after %d extra streams] events, fence per R/2", 2 * k + 1);
    run(nm, 2);
  }
  B = Bdef;
  return 0;
}
