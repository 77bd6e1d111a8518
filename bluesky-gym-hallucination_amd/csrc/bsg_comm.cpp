// bsg_comm.cpp -- the learner-row all-gather of the multi-GPU path as
// direct RCCL calls on a library-owned stream (include/bsg.h bsg_comm_*).
//
// Per RL step a shard's learner rows [n_local, obs+3] fp32 are all-gathered over xGMI into
// [world * n_local, obs+3] on every rank.  Through torch.distributed the host side of that
// gather cost ~35 us per step (c10d's enqueue ~28 us + Work.wait ~7 us,
// profiles/r03/shard_host_breakdown_k1.txt) against a 512-env shard's ~28 us kernel: one
// gather per step made the loop host-bound.  Here one call records an event on the
// caller's stream, makes the comm's own stream wait for it and enqueues ncclAllGather there.
// Completion is tracked by gather sequence number: a fence event is recorded behind every
// BSG_COMM_SLOTS/2-th gather, and bsg_comm_wait makes a stream wait for the oldest fence that
// covers the slot's last gather -- with a ring of BSG_COMM_SLOTS row buffers the step that
// next overwrites a slot finds its gather already covered by a fence its stream waited for,
// so that stream wait is issued once per BSG_COMM_SLOTS/2 steps instead of every step.
// The comm's stream has the greatest priority: one of the default priority may share a
// hardware queue with the caller's stream, which puts each gather between two steps.
// Measured (tools/probe/hostapi_probe.cpp with a 28 us kernel standing in for the 512-env
// shard, profiles/r04/comm/): 52.4 us per step with an event pair and a reverse wait every
// step on a default-priority stream (round 3's scheme), 35.6 us with the fences and the
// priority, 30.0 us for the launches alone; the product path (tools/shard_flag_sweep.py)
// 49.4 -> 33.4 us per step at 512 envs, 70.4 -> 55.6 at 4096.  (A completion value published
// by the step kernel's last workgroup instead of the event pair -- every workgroup counting
// itself out with a device-scope atomic -- tied at 512 envs and cost +58 us at 4096: the
// atomics on one address from 2,048 workgroups across eight XCDs serialise.)  All
// asynchronous.
// RCCL is resolved at run time: the librccl.so.1 the process already loaded (torch's) if
// any, else ROCm's.  One copy of RCCL per process, no link-time dependency.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "../../include/bsg.h"

namespace {

// the subset of rccl.h used here (ABI of /opt/rocm/include/rccl/rccl.h)
typedef struct ncclComm* ncclComm_t;
typedef struct { char internal[BSG_COMM_ID_BYTES]; } ncclUniqueId;
typedef int ncclResult_t;                 // ncclSuccess = 0
constexpr int kNcclFloat32 = 7;
constexpr int kNcclSum = 0, kNcclAvg = 4;   // ncclRedOp_t

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  // (optional: only bsg_comm_all_reduce needs it)
  ncclResult_t (*all_reduce)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_count)(ncclComm_t, int*) = nullptr;
  ncclResult_t (*comm_user_rank)(ncclComm_t, int*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string err;
};

thread_local std::string g_comm_err;

Rccl g_rccl;

std::string rccl_error_or_empty() { return g_rccl.err; }

Rccl* rccl() {
  Rccl& r = g_rccl;
  static bool tried = false;
  if (tried) return r.h ? &r : nullptr;
  tried = true;
  const char* names[] = {"librccl.so.1", "librccl.so"};
  for (const char* n : names)
    if ((r.h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;       // the process's copy (torch)
  if (!r.h) r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!r.h) {
    r.err = std::string("RCCL not found: ") + dlerror();
    return nullptr;
  }
  r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.h, "ncclGetUniqueId"));
  r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(r.h, "ncclCommInitRank"));
  r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(r.h, "ncclAllGather"));
  r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(r.h, "ncclAllReduce"));
  r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.h, "ncclCommDestroy"));
  r.comm_count = reinterpret_cast<decltype(r.comm_count)>(dlsym(r.h, "ncclCommCount"));
  r.comm_user_rank = reinterpret_cast<decltype(r.comm_user_rank)>(dlsym(r.h, "ncclCommUserRank"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.h, "ncclGetErrorString"));
  if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy || !r.comm_count ||
      !r.comm_user_rank) {
    r.err = "RCCL library lacks ncclGetUniqueId/ncclCommInitRank/ncclAllGather/ncclCommDestroy/"
            "ncclCommCount/ncclCommUserRank";
    r.h = nullptr;
    return nullptr;
  }
  return &r;
}

int comm_fail(int code, const std::string& msg) {
  g_comm_err = msg;
  return code;
}

std::string nccl_msg(Rccl* r, ncclResult_t e, const char* where) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), " (ncclResult %d)", e);
  return std::string(where) + ": " + (r->error_string ? r->error_string(e) : "") + buf;
}

}  // namespace

// A gather captured once as a HIP graph (one ncclAllGather node) and replayed: RCCL's own
// enqueue costs tens of us of host time per call (profiles/r04/shard_overhead_r04.txt), a
// graph launch a few.  Keyed by the buffers and size (the caller's ring of row blocks): the
// cache holds one graph per slot of the ring (a smaller FIFO cache would miss on every
// gather of the fused per-step path, which cycles through all BSG_COMM_SLOTS slots).
struct GatherGraph {
  const void* send = nullptr;
  void* recv = nullptr;
  int64_t count = -1;
  hipGraphExec_t exec = nullptr;
};
constexpr int kGraphCache = BSG_COMM_SLOTS;

constexpr int kFences = 4;              // fence events in flight (a ring)
constexpr int64_t kFenceEvery = BSG_COMM_SLOTS / 2;
constexpr int kWaited = 4;              // streams whose waited-for gather is remembered

struct bsg_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
  hipStream_t side = nullptr;           // the gathers' stream (greatest priority)
  hipEvent_t step_done[BSG_COMM_SLOTS] = {};   // caller-stream events (bsg_comm_all_gather)
  // gather g (1-based, in issue order) is covered by every fence recorded after it
  int64_t gseq = 0;                     // gathers issued
  int64_t slot_seq[BSG_COMM_SLOTS] = {};   // the last gather that read each slot (0: none)
  hipEvent_t fence[kFences] = {};
  int64_t fence_seq[kFences] = {};      // the gather each fence was recorded behind (0: none)
  int next_fence = 0;
  int64_t last_fence = 0;
  struct Waited { void* stream; int64_t seq; } waited[kWaited] = {};
  int next_waited = 0;
  bool use_graphs = false;              // BSG_COMM_GRAPHS=1: the gather as a replayed HIP graph
  GatherGraph graphs[kGraphCache];
  int next_graph = 0;
  int64_t graph_hits = 0, graph_captures = 0;
  int64_t reduces = 0;                  // bsg_comm_all_reduce calls
  // BSG_COMM_PROFILE=1: host time of each part of bsg_comm_all_gather, printed at destroy
  bool prof = false;
  double t_rec = 0, t_wait = 0, t_coll = 0, t_rec2 = 0;
  long n_calls = 0;
};

namespace {
inline double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

namespace {

// the graph of one ncclAllGather(send -> recv) on c->side, captured on first use
hipGraphExec_t gather_graph(bsg_comm* c, Rccl* r, const void* send, void* recv, int64_t count,
                            std::string* err) {
  for (auto& g : c->graphs)
    if (g.exec && g.send == send && g.recv == recv && g.count == count) {
      ++c->graph_hits;
      return g.exec;
    }
  ++c->graph_captures;
  GatherGraph& g = c->graphs[c->next_graph];
  c->next_graph = (c->next_graph + 1) % kGraphCache;
  if (g.exec) { (void)hipGraphExecDestroy(g.exec); g.exec = nullptr; }
  hipGraph_t graph = nullptr;
  hipError_t he = hipStreamBeginCapture(c->side, hipStreamCaptureModeThreadLocal);
  if (he != hipSuccess) { *err = std::string("hipStreamBeginCapture: ") + hipGetErrorString(he); return nullptr; }
  ncclResult_t e = r->all_gather(send, recv, (size_t)count, kNcclFloat32, c->nc, c->side);
  he = hipStreamEndCapture(c->side, &graph);
  if (e != 0) { *err = nccl_msg(r, e, "ncclAllGather (capture)"); if (graph) (void)hipGraphDestroy(graph); return nullptr; }
  if (he != hipSuccess) { *err = std::string("hipStreamEndCapture: ") + hipGetErrorString(he); return nullptr; }
  he = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (he != hipSuccess) { *err = std::string("hipGraphInstantiate: ") + hipGetErrorString(he); g.exec = nullptr; return nullptr; }
  g.send = send;
  g.recv = recv;
  g.count = count;
  return g.exec;
}

// the gather itself on c->side (a replayed graph or a plain ncclAllGather)
int enqueue_gather(bsg_comm* c, Rccl* r, const float* send, float* recv, int64_t count,
                   const char* who) {
  if (c->use_graphs) {
    std::string err;
    hipGraphExec_t ex = gather_graph(c, r, send, recv, count, &err);
    if (!ex) return comm_fail(BSG_E_HIP, std::string(who) + ": " + err);
    hipError_t he = hipGraphLaunch(ex, c->side);
    if (he != hipSuccess) return comm_fail(BSG_E_HIP, std::string("hipGraphLaunch: ") + hipGetErrorString(he));
    return BSG_OK;
  }
  ncclResult_t e = r->all_gather(send, recv, (size_t)count, kNcclFloat32, c->nc, c->side);
  if (e != 0) return comm_fail(BSG_E_HIP, nccl_msg(r, e, "ncclAllGather"));
  return BSG_OK;
}

// a fence event behind everything enqueued on c->side so far
int record_fence(bsg_comm* c) {
  const int k = c->next_fence;
  hipError_t he = hipEventRecord(c->fence[k], c->side);
  if (he != hipSuccess) return comm_fail(BSG_E_HIP, std::string("hipEventRecord(fence): ") + hipGetErrorString(he));
  c->fence_seq[k] = c->gseq;
  c->last_fence = c->gseq;
  c->next_fence = (k + 1) % kFences;
  return BSG_OK;
}

// bookkeeping after gather gseq + 1 read `slot`
int gathered(bsg_comm* c, int slot) {
  c->slot_seq[slot] = ++c->gseq;
  if (c->gseq - c->last_fence >= kFenceEvery) return record_fence(c);
  return BSG_OK;
}

int64_t* waited_mark(bsg_comm* c, void* stream) {
  for (auto& w : c->waited)
    if (w.stream == stream && w.seq > 0) return &w.seq;
  auto& w = c->waited[c->next_waited];
  c->next_waited = (c->next_waited + 1) % kWaited;
  w.stream = stream;
  w.seq = 0;
  return &w.seq;
}

// `stream` waits until gather `need` is complete: nothing if it already waited for a fence
// that covers it, else for the oldest fence that does (recorded now if none does yet)
int wait_for(bsg_comm* c, int64_t need, void* stream) {
  if (need <= 0) return BSG_OK;
  int64_t* w = waited_mark(c, stream);
  if (*w >= need) return BSG_OK;
  int best = -1;
  for (int k = 0; k < kFences; ++k)
    if (c->fence_seq[k] >= need && (best < 0 || c->fence_seq[k] < c->fence_seq[best])) best = k;
  if (best < 0) {
    if (int rc = record_fence(c)) return rc;
    best = (c->next_fence + kFences - 1) % kFences;
  }
  hipError_t he = hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), c->fence[best], 0);
  if (he != hipSuccess) return comm_fail(BSG_E_HIP, std::string("hipStreamWaitEvent: ") + hipGetErrorString(he));
  *w = c->fence_seq[best];
  return BSG_OK;
}

}  // namespace

extern "C" {

const char* bsg_comm_last_error(void) { return g_comm_err.c_str(); }

int32_t bsg_comm_unique_id(uint8_t* id) {
  if (!id) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_unique_id: null buffer");
  Rccl* r = rccl();
  if (!r) return comm_fail(BSG_E_UNSUPPORTED, "bsg_comm_unique_id: " + rccl_error_or_empty());
  ncclUniqueId u;
  ncclResult_t e = r->get_unique_id(&u);
  if (e != 0) return comm_fail(BSG_E_HIP, nccl_msg(r, e, "ncclGetUniqueId"));
  std::memcpy(id, u.internal, BSG_COMM_ID_BYTES);
  return BSG_OK;
}

int32_t bsg_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device,
                        bsg_comm** out) {
  if (!id || !out) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_create: null argument");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_create: rank out of range");
  Rccl* r = rccl();
  if (!r) return comm_fail(BSG_E_UNSUPPORTED, "bsg_comm_create: " + rccl_error_or_empty());
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) return comm_fail(BSG_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
  bsg_comm* c = new (std::nothrow) bsg_comm();
  if (!c) return comm_fail(BSG_E_STATE, "bsg_comm_create: out of host memory");
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclUniqueId u;
  std::memcpy(u.internal, id, BSG_COMM_ID_BYTES);
  ncclResult_t e = r->comm_init_rank(&c->nc, nranks, u, rank);
  if (e != 0) {
    delete c;
    return comm_fail(BSG_E_HIP, nccl_msg(r, e, "ncclCommInitRank"));
  }
  if (const char* gv = std::getenv("BSG_COMM_GRAPHS")) c->use_graphs = std::atoi(gv) != 0;
  if (const char* pv = std::getenv("BSG_COMM_PROFILE")) c->prof = std::atoi(pv) != 0;
  int least = 0, greatest = 0;
  he = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (he == hipSuccess) he = hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, greatest);
  for (int s = 0; s < BSG_COMM_SLOTS && he == hipSuccess; ++s)
    he = hipEventCreateWithFlags(&c->step_done[s], hipEventDisableTiming);
  for (int k = 0; k < kFences && he == hipSuccess; ++k)
    he = hipEventCreateWithFlags(&c->fence[k], hipEventDisableTiming);
  if (he != hipSuccess) {
    bsg_comm_destroy(c);
    return comm_fail(BSG_E_HIP, std::string("bsg_comm_create: ") + hipGetErrorString(he));
  }
  *out = c;
  return BSG_OK;
}

int32_t bsg_comm_destroy(bsg_comm* c) {
  if (!c) return BSG_OK;
  if (c->side) (void)hipStreamSynchronize(c->side);
  if (c->prof && c->n_calls > 0)
    std::fprintf(stderr, "bsg_comm profile: %ld calls, host us/call: event %.2f, stream wait %.2f, "
                 "collective %.2f (%s), fence bookkeeping %.2f\n", c->n_calls,
                 c->t_rec / c->n_calls, c->t_wait / c->n_calls, c->t_coll / c->n_calls,
                 c->use_graphs ? "graph launch" : "ncclAllGather", c->t_rec2 / c->n_calls);
  for (auto& g : c->graphs)
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
  for (int s = 0; s < BSG_COMM_SLOTS; ++s)
    if (c->step_done[s]) (void)hipEventDestroy(c->step_done[s]);
  for (int k = 0; k < kFences; ++k)
    if (c->fence[k]) (void)hipEventDestroy(c->fence[k]);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->nc) {
    if (Rccl* r = rccl()) r->comm_destroy(c->nc);
  }
  delete c;
  return BSG_OK;
}

int32_t bsg_comm_all_gather(bsg_comm* c, const float* send, float* recv, int64_t count,
                            int32_t slot, void* stream) {
  if (!c || !send || !recv) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_all_gather: null argument");
  if (slot < 0 || slot >= BSG_COMM_SLOTS || count < 0)
    return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_all_gather: slot or count out of range");
  Rccl* r = rccl();
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const double t0 = c->prof ? now_us() : 0.0;
  // the gather reads what the caller's stream wrote up to here (the step's learner rows)
  hipError_t he = hipEventRecord(c->step_done[slot], st);
  const double t1 = c->prof ? now_us() : 0.0;
  if (he == hipSuccess) he = hipStreamWaitEvent(c->side, c->step_done[slot], 0);
  const double t2 = c->prof ? now_us() : 0.0;
  if (he != hipSuccess) return comm_fail(BSG_E_HIP, std::string("bsg_comm_all_gather: ") + hipGetErrorString(he));
  if (int rc = enqueue_gather(c, r, send, recv, count, "bsg_comm_all_gather")) return rc;
  const double t3 = c->prof ? now_us() : 0.0;
  if (int rc = gathered(c, slot)) return rc;
  if (c->prof) {
    const double t4 = now_us();
    c->t_rec += t1 - t0; c->t_wait += t2 - t1; c->t_coll += t3 - t2; c->t_rec2 += t4 - t3;
    ++c->n_calls;
  }
  return BSG_OK;
}

int32_t bsg_comm_get_info(const bsg_comm* c, bsg_comm_info* out) {
  if (!c || !out) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_get_info: null argument");
  Rccl* r = rccl();
  if (!r || !c->nc) return comm_fail(BSG_E_STATE, "bsg_comm_get_info: no communicator");
  int n = 0, me = -1;
  ncclResult_t e = r->comm_count(c->nc, &n);
  if (e != 0) return comm_fail(BSG_E_HIP, nccl_msg(r, e, "ncclCommCount"));
  e = r->comm_user_rank(c->nc, &me);
  if (e != 0) return comm_fail(BSG_E_HIP, nccl_msg(r, e, "ncclCommUserRank"));
  out->nranks = n;
  out->rank = me;
  out->device = c->device;
  out->use_graphs = c->use_graphs ? 1 : 0;
  out->gathers = c->gseq;
  out->graph_hits = c->graph_hits;
  out->graph_captures = c->graph_captures;
  out->reduces = c->reduces;
  return BSG_OK;
}

// The learner's gradients: in place, on the caller's stream (no side stream, no events: the
// update that follows on that stream needs the result, and a graph capture of the update
// records the collective as one more node of the same stream)
int32_t bsg_comm_all_reduce(bsg_comm* c, float* buf, int64_t count, int32_t op, void* stream) {
  if (!c || !buf) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_all_reduce: null argument");
  if (count < 0 || (op != BSG_REDUCE_SUM && op != BSG_REDUCE_AVG))
    return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_all_reduce: count or op out of range");
  Rccl* r = rccl();
  if (!r || !c->nc) return comm_fail(BSG_E_STATE, "bsg_comm_all_reduce: no communicator");
  if (!r->all_reduce) return comm_fail(BSG_E_UNSUPPORTED, "bsg_comm_all_reduce: RCCL lacks ncclAllReduce");
  if (count == 0) return BSG_OK;
  ncclResult_t e = r->all_reduce(buf, buf, (size_t)count, kNcclFloat32,
                                 op == BSG_REDUCE_AVG ? kNcclAvg : kNcclSum, c->nc,
                                 reinterpret_cast<hipStream_t>(stream));
  if (e != 0) return comm_fail(BSG_E_HIP, nccl_msg(r, e, "ncclAllReduce"));
  ++c->reduces;
  return BSG_OK;
}

int32_t bsg_comm_wait(bsg_comm* c, int32_t slot, void* stream) {
  if (!c) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_wait: null comm");
  if (slot < 0 || slot >= BSG_COMM_SLOTS) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_wait: slot out of range");
  return wait_for(c, c->slot_seq[slot], stream);
}

}  // extern "C"
