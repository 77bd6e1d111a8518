// bsg_comm.cpp -- the learner-row all-gather of the multi-GPU path as
// direct RCCL calls on a library-owned stream (include/bsg.h bsg_comm_*).
//
// Per RL step a shard's learner rows [n_local, obs+3] fp32 are all-gathered over xGMI into
// [world * n_local, obs+3] on every rank.  Through torch.distributed the host side of that
// gather cost ~35 us per step (c10d's enqueue ~28 us + Work.wait ~7 us,
// profiles/r03/shard_host_breakdown_k1.txt) against a 512-env shard's ~28 us kernel: one
// gather per step made the loop host-bound.  Here one call records an event on the
// caller's stream, makes the comm's stream wait for it, enqueues ncclAllGather there and
// records the gather's completion per slot; bsg_comm_wait makes a stream wait for a slot's
// gather (the consumer, or the step that next overwrites those rows).  All asynchronous.
//
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

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
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
  r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.h, "ncclCommDestroy"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.h, "ncclGetErrorString"));
  if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy) {
    r.err = "RCCL library lacks ncclGetUniqueId/ncclCommInitRank/ncclAllGather/ncclCommDestroy";
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
// graph launch a few.  Keyed by the buffers and size (the caller's ring of row blocks).
struct GatherGraph {
  const void* send = nullptr;
  void* recv = nullptr;
  int64_t count = -1;
  hipGraphExec_t exec = nullptr;
};
constexpr int kGraphCache = 8;

struct bsg_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
  hipStream_t side = nullptr;           // the gathers' stream
  hipEvent_t step_done[BSG_COMM_SLOTS] = {};
  hipEvent_t gathered[BSG_COMM_SLOTS] = {};
  bool pending[BSG_COMM_SLOTS] = {};    // gathered[slot] recorded and not yet waited for
  bool use_graphs = true;               // BSG_COMM_GRAPHS=0: plain ncclAllGather per call
  GatherGraph graphs[kGraphCache];
  int next_graph = 0;
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
    if (g.exec && g.send == send && g.recv == recv && g.count == count) return g.exec;
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
  he = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  for (int s = 0; s < BSG_COMM_SLOTS && he == hipSuccess; ++s) {
    he = hipEventCreateWithFlags(&c->step_done[s], hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&c->gathered[s], hipEventDisableTiming);
  }
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
                 "collective %.2f (%s), event %.2f\n", c->n_calls, c->t_rec / c->n_calls,
                 c->t_wait / c->n_calls, c->t_coll / c->n_calls,
                 c->use_graphs ? "graph launch" : "ncclAllGather", c->t_rec2 / c->n_calls);
  for (auto& g : c->graphs)
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
  for (int s = 0; s < BSG_COMM_SLOTS; ++s) {
    if (c->step_done[s]) (void)hipEventDestroy(c->step_done[s]);
    if (c->gathered[s]) (void)hipEventDestroy(c->gathered[s]);
  }
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
  if (c->use_graphs) {
    std::string err;
    hipGraphExec_t ex = gather_graph(c, r, send, recv, count, &err);
    if (!ex) return comm_fail(BSG_E_HIP, "bsg_comm_all_gather: " + err);
    he = hipGraphLaunch(ex, c->side);
    if (he != hipSuccess) return comm_fail(BSG_E_HIP, std::string("hipGraphLaunch: ") + hipGetErrorString(he));
  } else {
    ncclResult_t e = r->all_gather(send, recv, (size_t)count, kNcclFloat32, c->nc, c->side);
    if (e != 0) return comm_fail(BSG_E_HIP, nccl_msg(r, e, "ncclAllGather"));
  }
  const double t3 = c->prof ? now_us() : 0.0;
  he = hipEventRecord(c->gathered[slot], c->side);
  if (he != hipSuccess) return comm_fail(BSG_E_HIP, std::string("bsg_comm_all_gather: ") + hipGetErrorString(he));
  if (c->prof) {
    const double t4 = now_us();
    c->t_rec += t1 - t0; c->t_wait += t2 - t1; c->t_coll += t3 - t2; c->t_rec2 += t4 - t3;
    ++c->n_calls;
  }
  c->pending[slot] = true;
  return BSG_OK;
}

int32_t bsg_comm_wait(bsg_comm* c, int32_t slot, void* stream) {
  if (!c) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_wait: null comm");
  if (slot < 0 || slot >= BSG_COMM_SLOTS) return comm_fail(BSG_E_INVALID_ARG, "bsg_comm_wait: slot out of range");
  if (!c->pending[slot]) return BSG_OK;      // nothing gathered into this slot yet
  hipError_t he = hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), c->gathered[slot], 0);
  if (he != hipSuccess) return comm_fail(BSG_E_HIP, std::string("bsg_comm_wait: ") + hipGetErrorString(he));
  return BSG_OK;
}

}  // extern "C"
