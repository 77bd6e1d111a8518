// bsg_abi.cpp -- extern "C" boundary of libbsg.so (declared in include/bsg.h).
//
// Validation, thread-local error reporting and launch plumbing only; all arithmetic
// lives in bsg_kernels.hip.  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/bsg.h"
#include "bsg_areas.h"
#include "bsg_internal.h"

struct bsg_ctx {
  bsg_config cfg;
  bsg_buffers bufs;
  bool bound = false;
  int obs_dim = 0;
  int spawn_width = 0;
  bsg::Route route{};
  bsg::RouteTrig route_t{};
  bsg::WindDev wind{};
  // optional per-launch timing (bsg_set_timing): an event pair around every
  // `timing`-th launch (0 = off)
  int timing = 0;
  long long launch_count = 0;
  unsigned long long* stamps = nullptr;
  unsigned lds_pad = 0;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double folded_ms = 0.0;          // timed launches already folded out of `pending`
  int folded_n = 0;
  // lookahead scratch (bsg_set_lookahead): slot parity, tag generation, and what the next
  // launch must re-initialise first (la_dirty: the scratch; memo_dirty: the caller's
  // memo_cache, whose intruder entries the main workgroups do not keep current while the
  // lookahead runs)
  double* la = nullptr;
  int la_par = 0;
  uint32_t la_gen = 0;
  uint32_t la_seq = 0;              // launches since the last re-arm (snapshot parity)
  bool la_dirty = false, memo_dirty = false, la_was_active = false;
  bool la_prime = false;            // the next launch runs the priming pass first
  // a launch was captured into a HIP graph: the host-side slot / snapshot parities cannot
  // follow the graph's replays, so this ctx runs without the lookahead from then on
  bool la_captured = false;
  int no_fastpath = 0;
  // Merge's creation-state constants (KParams::spawn_k), computed once by the first launch
  // outside a stream capture: 0 = not yet, 1 = valid, -1 = unavailable
  int spawn_k_state = 0;
  double spawn_k[8] = {};
  double* spawn_k_dev = nullptr;
  // the env module's constants (bsg_set_params; Merge: merge_env.py:13-46)
  double kp[BSG_MERGE_NPARAMS] = {15.0, 20.0, 4.0, 10.0, 1.0, -0.1, -1.0, 50.0, 200.0, 20.0, 500.0};
  bool launched = false;            // a reset / step has been enqueued
  // trajectory store (bsg_set_trajectory; bsg_internal.h tj_doubles): the producers run on
  // their own stream of the least priority, at most kProdMax launches enqueued (they run one
  // after the other); each publishes itself on the device when its last wave ends
  // (produce_kernel), so the step launches enqueued ahead of it see it as soon as it is done
  double* traj = nullptr;
  bool traj_sync = false;           // test hook: producers on the caller's stream, in order
  bool traj_noasync = false;        // BSG_TRAJ_NOASYNC=1 (A/B runs): reset-time production only
  int traj_wprio = 1;               // BSG_TRAJ_WPRIO=1: producer waves at s_setprio 1 (else 0)
  int traj_every = 1;               // BSG_TRAJ_EVERY: step launches between producer launches
  int traj_sleep = 0;               // BSG_TRAJ_SLEEP: produce_kernel prod_sleep
  uint32_t traj_gen = 1;            // 1..0xFFE; bumped when the stored episodes may be stale
  int prod_out = 0;                 // producer launches enqueued and not seen complete
  int prod_head = 0;                // oldest of them in ev_prod[] (a ring)
  int steps_since_prod = 0;
  int64_t prod_launches = 0;
  hipStream_t prod_st = nullptr;
  hipEvent_t ev_step = nullptr;
  hipEvent_t ev_prod[4] = {};
};

namespace {

thread_local std::string g_err;

__attribute__((format(printf, 2, 3))) int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return BSG_E_HIP;
}

hipEvent_t take_event(bsg_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// sorted-key position of wind_u among the env kind's observation keys (wind.py:18-24 adds
// wind_u/wind_v; gymnasium spaces.Dict sorts): right before the first key > "wind_v"
int wind_obs_pos(const bsg_config& cfg) {
  const int K = cfg.num_ac_state, NI = cfg.num_ac - 1;
  switch (cfg.env_kind) {
    case BSG_ENV_MERGE: return 5 + 5 * K;          // ... waypoint_dist | x_r, y_r
    case BSG_ENV_VERTICAL_CR: return 4 + 4 * NI;   // ... vz | x_/y_/z_difference_speed
    case BSG_ENV_DESCENT: return 4;                 // all keys sort before "wind"
    case BSG_ENV_HORIZONTAL_CR: return 3 * NI + 3; // ... waypoint_distance | x_/y_...
    case BSG_ENV_STATIC_OBSTACLE: return 3 + 4 * bsg::SO_NOBST;  // all keys sort before "wind"
    case BSG_ENV_SECTOR_CR: return 3 + 5 * K;      // ... vx_r, vy_r | x_r, y_r
    case BSG_ENV_PLAN_WAYPOINT: return 4 * bsg::PW_NWPT;  // ... waypoint_reached | (end)
    default: return 0;
  }
}

bool la_active(const bsg_ctx* c);

bsg::KParams make_params(const bsg_ctx* c, int mode) {
  bsg::KParams p;
  std::memset(&p, 0, sizeof(p));
  p.cfg = c->cfg;
  p.route = c->route;
  p.route_t = c->route_t;
  p.b = c->bufs;
  p.mode = mode;
  p.E = c->cfg.num_envs;
  p.N = c->cfg.num_ac;
  p.K = c->cfg.num_ac_state;
  p.obs_dim = c->obs_dim;
  p.spawn_width = c->spawn_width;
  p.seed = c->cfg.seed;
  p.stamps = c->stamps;
  p.lds_pad = c->lds_pad;
  p.wind = c->wind;
  p.wpos = wind_obs_pos(c->cfg);
  p.la = la_active(c) ? c->la : nullptr;
  p.la_par = c->la_par;
  p.la_gen = c->la_gen;
  p.la_seq = c->la_seq;
  p.no_fastpath = c->no_fastpath;
  p.spawn_k_ok = c->spawn_k_state == 1 ? 1 : 0;
  for (int k = 0; k < 8; ++k) p.spawn_k[k] = c->spawn_k[k];
  for (int k = 0; k < BSG_MERGE_NPARAMS; ++k) p.kp[k] = c->kp[k];
  p.traj_gen = c->traj_gen;
  p.traj_S = c->cfg.max_episode_steps;
  return p;
}

// KParams::spawn_k (Merge): one small kernel and a read-back, once per ctx, by the first
// launch that is not being captured into a graph; BSG_NO_FASTPATH=1 leaves it off (the
// tests compare the two)
int spawn_k_prepare(bsg_ctx* c, hipStream_t st) {
  if (c->spawn_k_state != 0) return BSG_OK;
  if (c->cfg.env_kind != BSG_ENV_MERGE || c->no_fastpath) { c->spawn_k_state = -1; return BSG_OK; }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipError_t e = hipStreamIsCapturing(st, &cs);
  if (e != hipSuccess) return hip_fail(e, "hipStreamIsCapturing");
  if (cs != hipStreamCaptureStatusNone) return BSG_OK;          // (a later launch does it)
  c->spawn_k_state = -1;
  if (!c->spawn_k_dev && (e = hipMalloc(reinterpret_cast<void**>(&c->spawn_k_dev), 8 * sizeof(double))) != hipSuccess)
    return hip_fail(e, "hipMalloc(spawn_k)");
  double h[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  const double spd = c->cfg.kind_option > 0 ? (double)c->cfg.kind_option : 100.0;   // spawn_merge
  if ((e = bsg::spawn_consts_merge(spd, 10000.0, c->spawn_k_dev, st)) != hipSuccess)
    return hip_fail(e, "spawn constants launch");
  if ((e = hipMemcpyAsync(h, c->spawn_k_dev, sizeof(h), hipMemcpyDeviceToHost, st)) != hipSuccess)
    return hip_fail(e, "hipMemcpyAsync(spawn_k)");
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  if (h[4] == 1.0) {
    for (int k = 0; k < 8; ++k) c->spawn_k[k] = h[k];
    c->spawn_k_state = 1;
  }
  return BSG_OK;
}

// the lookahead runs for a bound Merge / Vertical scratch without a wind field
// (bsg_set_lookahead refuses the configurations it cannot serve: other kinds, SAME_STEP
// autoreset) and never for a ctx whose launches were captured into a graph
bool la_active(const bsg_ctx* c) {
  return c->la != nullptr && c->wind.np == 0 && !c->la_captured;
}

size_t la_bytes(const bsg_config& cfg) {
  return 8 * bsg::la_doubles((size_t)cfg.num_envs, (size_t)cfg.num_ac);
}

// Before a launch: re-initialise what a lookahead transition left stale (0xFF bytes = a
// NaN double: a memo miss / a tag no generation produces), on the launch stream.
int la_prepare(bsg_ctx* c, hipStream_t st) {
  const bool act = la_active(c);
  if (act != c->la_was_active) {
    c->la_dirty = c->la_dirty || act;
    c->memo_dirty = true;
    c->la_was_active = act;
  }
  if (c->memo_dirty && c->bufs.memo_cache) {
    // Not into a graph: a launch being captured turns the lookahead off (la_captured), and
    // at that on -> off transition the cache needs no reset -- the intruder entries were
    // invalidated when the lookahead came on and never written since (its blocks keep their
    // own memo), the ownship entries stayed current.  A reset captured into the graph
    // measured inexact replays (tests/test_gpu_lookahead.py
    // ::test_lookahead_off_once_a_launch_is_captured, profiles/r04/capture_replay.txt); the
    // flag stays set, so the next launch outside a graph resets the cache as before.
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipError_t e = hipStreamIsCapturing(st, &cs);
    if (e != hipSuccess) return hip_fail(e, "hipStreamIsCapturing");
    if (cs != hipStreamCaptureStatusNone) return BSG_OK;
    const size_t EN = (size_t)c->cfg.num_envs * c->cfg.num_ac;
    e = hipMemsetAsync(c->bufs.memo_cache, 0xFF, 8 * (2 * EN + 4 * (size_t)c->cfg.num_envs), st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(memo_cache)");
  }
  c->memo_dirty = false;
  if (act && c->la_dirty) {
    hipError_t e = hipMemsetAsync(c->la, 0xFF, la_bytes(c->cfg), st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(lookahead)");
    c->la_gen = (c->la_gen % 0x7ffe) + 1;
    c->la_par = 0;
    c->la_seq = 0;
    c->la_dirty = false;
    c->la_prime = true;
  }
  return BSG_OK;
}

// A caller that enables timing and never polls bsg_step_timing must not grow `pending`
// (and live hipEvents) without bound: past kMaxPending pairs, completed pairs are folded
// into running totals and their events recycled; if none has completed, the oldest is
// waited for.
constexpr size_t kMaxPending = 1024;

// Folds one pair into the running totals and recycles its events; on failure the pair is
// left alone (still the caller's to keep in `pending`).
int fold_pair(bsg_ctx* c, std::pair<hipEvent_t, hipEvent_t> pr) {
  hipError_t e = hipEventSynchronize(pr.second);
  if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
  float ms = 0.f;
  e = hipEventElapsedTime(&ms, pr.first, pr.second);
  if (e != hipSuccess) return hip_fail(e, "hipEventElapsedTime");
  c->folded_ms += ms;
  ++c->folded_n;
  c->ev_pool.push_back(pr.first);
  c->ev_pool.push_back(pr.second);
  return BSG_OK;
}

int trim_pending(bsg_ctx* c) {
  if (c->pending.size() < kMaxPending) return BSG_OK;
  size_t keep = 0;
  for (size_t i = 0; i < c->pending.size(); ++i) {
    if (hipEventQuery(c->pending[i].second) == hipSuccess) {
      if (int r = fold_pair(c, c->pending[i])) {
        // drop the pairs already folded (their events are back in the pool); keep the
        // failing one and the unvisited tail
        c->pending.erase(c->pending.begin() + keep, c->pending.begin() + i);
        return r;
      }
    } else {
      c->pending[keep++] = c->pending[i];
    }
  }
  c->pending.resize(keep);
  if (keep >= kMaxPending) {            // nothing finished yet: wait for the oldest
    if (int r = fold_pair(c, c->pending.front())) return r;
    c->pending.erase(c->pending.begin());
  }
  return BSG_OK;
}

// ---- trajectory store scheduling ------------------------------------------------------

constexpr int kProdMax = 2;         // producer launches enqueued at once (<= 4)

// wait for the enqueued producers (their buffers are about to change or go away)
int traj_quiesce(bsg_ctx* c) {
  if (!c->prod_out) return BSG_OK;
  hipError_t e = hipStreamSynchronize(c->prod_st);
  if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize(producer)");
  c->prod_out = 0;
  return BSG_OK;
}

// retire the producer launches that have completed (flow control only: publication is the
// producers' own, on the device)
void traj_poll(bsg_ctx* c) {
  while (c->prod_out > 0 && hipEventQuery(c->ev_prod[c->prod_head]) == hipSuccess) {
    c->prod_head = (c->prod_head + 1) % 4;
    --c->prod_out;
  }
}

void traj_new_gen(bsg_ctx* c) {
  c->traj_gen = (c->traj_gen % 0xFFEu) + 1u;
}

// Before a launch: retire the stored episodes when this launch spawns from host rows (the
// store holds Philox episodes: a host-row episode under the same counter is another one)
int traj_before(bsg_ctx* c, hipStream_t st, const double* spawn) {
  (void)st;
  traj_poll(c);
  if (spawn) traj_new_gen(c);
  return BSG_OK;
}

// After a launch: a reset with device spawns flies the episodes it just created and the next
// ones on this stream (ordered: usable from the next launch on); a step launch starts the
// next producer launch on the producer stream when none is in flight
int traj_after(bsg_ctx* c, const bsg::KParams& p0, hipStream_t st, int mode, const double* spawn) {
  bsg::KParams q = p0;
  q.actions = nullptr;
  q.spawn = nullptr;
  hipError_t e;
  if (mode == bsg::MODE_RESET) {
    if (spawn) return BSG_OK;
    // (the producer memo regions are per episode-ahead d: no two producer launches at once)
    if (int r = traj_quiesce(c)) return r;
    q.prod_d0 = 0;
    q.prod_d1 = 2;
    q.prod_q = bsg::TJ_SMAX;          // whole episodes
    q.prod_async = 0;
    if ((e = bsg::launch_produce(q, st)) != hipSuccess) return hip_fail(e, "produce launch (reset)");
    ++c->prod_launches;
    c->steps_since_prod = 1 << 20;
    return BSG_OK;
  }
  if (mode != bsg::MODE_STEP || c->prod_out >= kProdMax || c->traj_noasync ||
      ++c->steps_since_prod < c->traj_every)
    return BSG_OK;
  c->steps_since_prod = 0;
  q.env_mask = nullptr;
  q.prod_d0 = 0;                    // (the running episode: continued only)
  q.prod_d1 = bsg::TJ_D;
  q.prod_q = bsg::TJ_SMAX;
  q.is_prod = c->traj_wprio == 1 ? 2 : 1;
  q.prod_sleep = c->traj_sleep;
  q.prod_async = 1;                 // (the running episode continued only, also in sync mode)
  if (c->traj_sync) {
    if ((e = bsg::launch_produce(q, st)) != hipSuccess) return hip_fail(e, "produce launch");
    ++c->prod_launches;
    return BSG_OK;
  }
  q.prod_async = 1;
  if ((e = hipEventRecord(c->ev_step, st)) != hipSuccess) return hip_fail(e, "hipEventRecord(step)");
  if ((e = hipStreamWaitEvent(c->prod_st, c->ev_step, 0)) != hipSuccess)
    return hip_fail(e, "hipStreamWaitEvent(producer stream)");
  if ((e = bsg::launch_produce(q, c->prod_st)) != hipSuccess) return hip_fail(e, "produce launch");
  const int slot = (c->prod_head + c->prod_out) % 4;
  if ((e = hipEventRecord(c->ev_prod[slot], c->prod_st)) != hipSuccess)
    return hip_fail(e, "hipEventRecord(producer)");
  ++c->prod_out;
  ++c->prod_launches;
  return BSG_OK;
}

int launch(bsg_ctx* c, int mode, const double* actions, const double* spawn,
           const uint8_t* env_mask, void* stream) {
  hipError_t e = hipSetDevice(c->cfg.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (c->la && !c->la_captured) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    e = hipStreamIsCapturing(st, &cs);
    if (e != hipSuccess) return hip_fail(e, "hipStreamIsCapturing");
    if (cs != hipStreamCaptureStatusNone) c->la_captured = true;
  }
  if (int r = la_prepare(c, st)) return r;
  if (int r = spawn_k_prepare(c, st)) return r;
  // trajectory store: active with the lookahead itself (no wind, no graph capture)
  const bool tj = c->traj && la_active(c);
  // (an in-flight producer writes only the store; a launch without it leaves it running --
  // synchronising here would be illegal inside a stream capture)
  if (tj) {
    if (int r = traj_before(c, st, spawn)) return r;
  }
  bsg::KParams p = make_params(c, mode);
  p.actions = actions;
  p.spawn = spawn;
  p.env_mask = env_mask;
  p.traj = tj ? c->traj : nullptr;
  c->launched = true;
#if defined(BSG_LA_LEGACY) && BSG_LA_LEGACY
  c->la_prime = false;                // negative-control debug builds: round 3 had no priming pass
#endif
  if (p.la && c->la_prime) {
    // after a re-arm: from the state the previous launch finished writing, the slot and the
    // env-scalar snapshot this launch's lookahead waves read (bsg_kernels.hip lookahead_role)
    bsg::KParams q = p;
    q.mode = bsg::MODE_PRIME;
    q.actions = nullptr;
    q.spawn = nullptr;
    q.env_mask = nullptr;
    e = bsg::launch_step(q, st);
    if (e != hipSuccess) return hip_fail(e, "lookahead priming launch");
    c->la_prime = false;
  }
  hipEvent_t t0 = nullptr, t1 = nullptr;
  const bool timed = c->timing > 0 && (c->launch_count++ % c->timing) == 0;
  if (timed) {
    if (int r = trim_pending(c)) return r;
    t0 = take_event(c);
    t1 = take_event(c);
    if (!t0 || !t1) {
      if (t0) c->ev_pool.push_back(t0);
      if (t1) c->ev_pool.push_back(t1);
      return fail(BSG_E_HIP, "hipEventCreate failed");
    }
    if ((e = hipEventRecord(t0, st)) != hipSuccess) {
      c->ev_pool.push_back(t0);
      c->ev_pool.push_back(t1);
      return hip_fail(e, "hipEventRecord");
    }
  }
  e = bsg::launch_step(p, st);
  if (e != hipSuccess) {
    if (timed) { c->ev_pool.push_back(t0); c->ev_pool.push_back(t1); }
    return hip_fail(e, "kernel launch");
  }
  if (timed) {
    if ((e = hipEventRecord(t1, st)) != hipSuccess) {
      c->ev_pool.push_back(t0);
      c->ev_pool.push_back(t1);
      return hip_fail(e, "hipEventRecord");
    }
    c->pending.emplace_back(t0, t1);
  }
  if (p.la) {
    if (mode == bsg::MODE_STEP) c->la_par ^= 1;   // this step wrote the other slot
    ++c->la_seq;                                   // and the other snapshot
  }
  if (tj) return traj_after(c, p, st, mode, spawn);
  return BSG_OK;
}

}  // namespace

extern "C" {

int32_t bsg_abi_version(void) { return BSG_ABI_VERSION; }

const char* bsg_last_error(void) { return g_err.c_str(); }

int32_t bsg_obs_dim(int32_t kind, int32_t num_ac, int32_t k) {
  switch (kind) {
    case BSG_ENV_MERGE: return (num_ac >= 2 && k >= 1 && k <= num_ac - 1) ? 5 + 7 * k : BSG_E_INVALID_ARG;
    case BSG_ENV_VERTICAL_CR: return num_ac >= 2 ? 4 + 7 * (num_ac - 1) : BSG_E_INVALID_ARG;
    case BSG_ENV_DESCENT: return num_ac == 1 ? 4 : BSG_E_INVALID_ARG;
    case BSG_ENV_HORIZONTAL_CR: return num_ac >= 2 ? 3 + 5 * (num_ac - 1) : BSG_E_INVALID_ARG;
    case BSG_ENV_STATIC_OBSTACLE: return num_ac == 1 ? 3 + 4 * bsg::SO_NOBST : BSG_E_INVALID_ARG;
    case BSG_ENV_SECTOR_CR:        // at least NUM_AC_STATE + 1 aircraft (sector_cr_env.py:97)
      return (num_ac >= 5 && k >= 1 && k <= 4) ? 3 + 7 * k : BSG_E_INVALID_ARG;
    case BSG_ENV_PLAN_WAYPOINT: return num_ac == 1 ? 4 * bsg::PW_NWPT : BSG_E_INVALID_ARG;
    default: return BSG_E_INVALID_ARG;
  }
}

int32_t bsg_action_dim(int32_t kind) {
  switch (kind) {
    case BSG_ENV_MERGE:
    case BSG_ENV_STATIC_OBSTACLE:
    case BSG_ENV_SECTOR_CR: return 2;
    case BSG_ENV_VERTICAL_CR:
    case BSG_ENV_DESCENT:
    case BSG_ENV_HORIZONTAL_CR:
    case BSG_ENV_PLAN_WAYPOINT: return 1;
    default: return BSG_E_INVALID_ARG;
  }
}

int32_t bsg_spawn_width(int32_t kind, int32_t num_ac) {
  switch (kind) {
    case BSG_ENV_MERGE: return 2 * num_ac;
    case BSG_ENV_VERTICAL_CR: return 2 + 4 * (num_ac - 1);
    case BSG_ENV_DESCENT: return 2;
    case BSG_ENV_HORIZONTAL_CR: return 3 * (num_ac - 1) + 1;
    case BSG_ENV_STATIC_OBSTACLE: return bsg::SO_SPAWN_W;
    case BSG_ENV_SECTOR_CR: return 4 + 2 * bsg::SC_VMAX + 3 * num_ac;
    case BSG_ENV_PLAN_WAYPOINT: return 2 * bsg::PW_NWPT;
    default: return BSG_E_INVALID_ARG;
  }
}

int32_t bsg_geom_width(int32_t kind, int32_t num_ac) {
  (void)num_ac;
  switch (kind) {
    case BSG_ENV_STATIC_OBSTACLE: return bsg::SO_GEOM;
    case BSG_ENV_SECTOR_CR: return bsg::SC_GEOM;
    case BSG_ENV_PLAN_WAYPOINT: return bsg::PW_GEOM;
    default: return 0;
  }
}

int32_t bsg_create(const bsg_config* cfg, bsg_ctx** out) {
  if (!cfg || !out) return fail(BSG_E_INVALID_ARG, "bsg_create: null argument");
  *out = nullptr;
  if (cfg->abi_version != BSG_ABI_VERSION)
    return fail(BSG_E_INVALID_ARG, "bsg_create: abi_version mismatch (got %lld)", (long long)(cfg->abi_version));
  if (cfg->num_envs <= 0) return fail(BSG_E_INVALID_ARG, "bsg_create: num_envs must be > 0");
  if (cfg->num_ac < 1 || cfg->num_ac > BSG_MAX_AC)
    return fail(BSG_E_INVALID_ARG, "bsg_create: num_ac must be in [1, 64] (got %lld)", (long long)(cfg->num_ac));
  const int od = bsg_obs_dim(cfg->env_kind, cfg->num_ac, cfg->num_ac_state);
  if (od < 0) return fail(BSG_E_INVALID_ARG, "bsg_create: invalid env_kind/num_ac/num_ac_state");
  if (cfg->action_frequency < 0) return fail(BSG_E_INVALID_ARG, "bsg_create: action_frequency < 0");
  if (!(cfg->simdt > 0.0)) return fail(BSG_E_INVALID_ARG, "bsg_create: simdt must be > 0");
  if (cfg->autoreset_mode < 0 || cfg->autoreset_mode > 2)
    return fail(BSG_E_INVALID_ARG, "bsg_create: invalid autoreset_mode");
  if (cfg->route_len < 0 || cfg->route_len > BSG_MAX_ROUTE)
    return fail(BSG_E_INVALID_ARG, "bsg_create: route_len out of range");
  if (cfg->env_offset < 0) return fail(BSG_E_INVALID_ARG, "bsg_create: env_offset < 0");
  if (cfg->kind_option != 0 && !(cfg->env_kind == BSG_ENV_SECTOR_CR && cfg->kind_option == 1) &&
      !(cfg->env_kind == BSG_ENV_MERGE && cfg->kind_option > 0 && cfg->kind_option <= 400))
    return fail(BSG_E_INVALID_ARG, "bsg_create: invalid kind_option (%lld)", (long long)(cfg->kind_option));
  if (cfg->env_kind == BSG_ENV_MERGE && cfg->route_len < 1)
    return fail(BSG_E_INVALID_ARG, "bsg_create: Merge needs the FIX/RWY route");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  if (cfg->device < 0 || cfg->device >= ndev)
    return fail(BSG_E_INVALID_ARG, "bsg_create: device ordinal out of range (%lld)", (long long)(cfg->device));
  bsg_ctx* c = new (std::nothrow) bsg_ctx();
  if (!c) return fail(BSG_E_STATE, "bsg_create: out of host memory");
  c->cfg = *cfg;
  c->obs_dim = od;
  c->spawn_width = bsg_spawn_width(cfg->env_kind, cfg->num_ac);
  c->route.len = cfg->route_len;
  for (int k = 0; k < BSG_MAX_ROUTE; ++k) {
    c->route.lat[k] = cfg->route_lat[k];
    c->route.lon[k] = cfg->route_lon[k];
    c->route.next_qdr[k] = cfg->route_next_qdr[k];
    // geo.rwgs84 of the waypoint latitude (the LNAV distance bounds' centre)
    const double lat = cfg->route_lat[k] * (3.141592653589793 / 180.0);
    const double a = 6378137.0, b = 6356752.314245;
    const double an = a * a * std::cos(lat), bn = b * b * std::sin(lat);
    const double ad = a * std::cos(lat), bd = b * std::sin(lat);
    c->route.rwgs[k] = std::sqrt((an * an + bn * bn) / (ad * ad + bd * bd));
    bsg::sincos_t(cfg->route_lat[k] * bsg::kD2R, &c->route_t.sinlat[k], &c->route_t.coslat[k]);
    c->route_t.lonr[k] = cfg->route_lon[k] * bsg::kD2R;
    c->route_t.pnq[k] = bsg::pymod360(cfg->route_next_qdr[k]);
  }
  if (const char* pad = std::getenv("BSG_LDS_PAD_BYTES")) c->lds_pad = (unsigned)std::atoi(pad);
  if (const char* nf = std::getenv("BSG_NO_FASTPATH")) c->no_fastpath = std::atoi(nf) != 0;
  *out = c;
  return BSG_OK;
}

int32_t bsg_set_params(bsg_ctx* c, const double* v, int32_t n) {
  if (!c || !v) return fail(BSG_E_INVALID_ARG, "bsg_set_params: null argument");
  if (c->cfg.env_kind != BSG_ENV_MERGE)
    return fail(BSG_E_UNSUPPORTED, "bsg_set_params: MergeEnv only");
  if (n != BSG_MERGE_NPARAMS)
    return fail(BSG_E_INVALID_ARG, "bsg_set_params: %d values, MergeEnv takes %d", (int)n,
                (int)BSG_MERGE_NPARAMS);
  if (c->launched)
    return fail(BSG_E_STATE, "bsg_set_params: the ctx has launched already");
  for (int k = 0; k < n; ++k)
    if (!std::isfinite(v[k])) return fail(BSG_E_INVALID_ARG, "bsg_set_params: value %d not finite", k);
  if (!(v[BSG_MP_D_HEADING] >= 0.0) || !(v[BSG_MP_SPAWN_DISTANCE_MIN] >= 0.0) ||
      !(v[BSG_MP_SPAWN_DISTANCE_MIN] <= v[BSG_MP_SPAWN_DISTANCE_MAX]) ||
      !(v[BSG_MP_INTRUDER_DISTANCE_MIN] >= 0.0) ||
      !(v[BSG_MP_INTRUDER_DISTANCE_MIN] <= v[BSG_MP_INTRUDER_DISTANCE_MAX]))
    return fail(BSG_E_INVALID_ARG, "bsg_set_params: D_HEADING < 0 or a distance range out of order");
  for (int k = 0; k < n; ++k) c->kp[k] = v[k];
  return BSG_OK;
}

int32_t bsg_destroy(bsg_ctx* c) {
  if (!c) return BSG_OK;
  (void)traj_quiesce(c);
  if (c->prod_st) (void)hipStreamSynchronize(c->prod_st);
  if (c->ev_step) (void)hipEventDestroy(c->ev_step);
  for (auto ev : c->ev_prod)
    if (ev) (void)hipEventDestroy(ev);
  if (c->prod_st) (void)hipStreamDestroy(c->prod_st);
  for (auto& pr : c->pending) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  for (auto ev : c->ev_pool) (void)hipEventDestroy(ev);
  if (c->spawn_k_dev) (void)hipFree(c->spawn_k_dev);
  delete c;
  return BSG_OK;
}

int32_t bsg_bind(bsg_ctx* c, const bsg_buffers* b) {
  if (!c || !b) return fail(BSG_E_INVALID_ARG, "bsg_bind: null argument");
  const void* required[] = {b->lat, b->lon, b->alt, b->hdg, b->tas, b->cas, b->vs, b->ax,
                            b->ap_trk, b->selspd, b->selalt, b->selvs, b->nav,
                            b->step_count, b->flags, b->episode, b->wpt_reach, b->faf_reached,
                            b->total_intrusions, b->total_reward, b->drift_sum, b->target_alt,
                            b->final_altitude, b->obs, b->reward, b->terminated, b->truncated};
  for (size_t i = 0; i < sizeof(required) / sizeof(required[0]); ++i)
    if (!required[i]) return fail(BSG_E_INVALID_ARG, "bsg_bind: required buffer #%lld is NULL", (long long)i);
  if (c->cfg.env_kind == BSG_ENV_HORIZONTAL_CR && (!b->env_wpt_lat || !b->env_wpt_lon))
    return fail(BSG_E_INVALID_ARG, "bsg_bind: HorizontalCR needs env_wpt_lat/env_wpt_lon");
  if (bsg_geom_width(c->cfg.env_kind, c->cfg.num_ac) > 0 && !b->env_geom)
    return fail(BSG_E_INVALID_ARG, "bsg_bind: StaticObstacle/SectorCR/PlanWaypoint need env_geom");
  if (c->cfg.env_kind == BSG_ENV_STATIC_OBSTACLE && !b->env_aux)
    return fail(BSG_E_INVALID_ARG, "bsg_bind: StaticObstacle needs env_aux");
  if (c->cfg.env_kind == BSG_ENV_MERGE && !b->topk)
    return fail(BSG_E_INVALID_ARG, "bsg_bind: Merge needs topk");
  if (c->cfg.autoreset_mode == BSG_AUTORESET_SAME_STEP && !b->final_obs)
    return fail(BSG_E_INVALID_ARG, "bsg_bind: SAME_STEP autoreset needs final_obs");
  if (c->wind.np > 0 && (!b->gs || !b->trk))
    return fail(BSG_E_INVALID_ARG, "bsg_bind: a wind field needs gs/trk");
  if (c->cfg.compute_cd && c->cfg.num_ac > 1 &&
      (!b->conf_mask || !b->los_mask || !b->tcpamax || !b->min_sep))
    return fail(BSG_E_INVALID_ARG, "bsg_bind: compute_cd needs conf_mask/los_mask/tcpamax/min_sep");
  if (int r = traj_quiesce(c)) return r;       // (it reads the episode words of the old buffers)
  c->bufs = *b;
  c->bound = true;
  c->la_dirty = true;               // new buffers: the lookahead restarts from them
  traj_new_gen(c);
  return BSG_OK;
}

int64_t bsg_lookahead_bytes(const bsg_ctx* c) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_lookahead_bytes: null ctx");
  if ((c->cfg.env_kind != BSG_ENV_MERGE && c->cfg.env_kind != BSG_ENV_VERTICAL_CR) ||
      c->cfg.autoreset_mode == BSG_AUTORESET_SAME_STEP)
    return 0;
  return (int64_t)la_bytes(c->cfg);
}

int32_t bsg_set_lookahead(bsg_ctx* c, void* scratch, int64_t bytes) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_set_lookahead: null ctx");
  if (scratch) {
    if (bsg_lookahead_bytes(c) == 0)
      return fail(BSG_E_UNSUPPORTED, "bsg_set_lookahead: MergeEnv / VerticalCREnv with NEXT_STEP "
                  "or no autoreset only");
    if (bytes < (int64_t)la_bytes(c->cfg))
      return fail(BSG_E_INVALID_ARG, "bsg_set_lookahead: scratch too small (need %lld bytes)",
                  (long long)la_bytes(c->cfg));
    if (reinterpret_cast<uintptr_t>(scratch) & 7)
      return fail(BSG_E_INVALID_ARG, "bsg_set_lookahead: scratch must be 8-byte aligned");
  }
  if (int r = traj_quiesce(c)) return r;
  c->la = static_cast<double*>(scratch);
  c->la_dirty = true;               // also re-arms after the caller wrote state directly
  traj_new_gen(c);
  return BSG_OK;
}

int64_t bsg_trajectory_bytes(const bsg_ctx* c) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_trajectory_bytes: null ctx");
#if (defined(BSG_LA_WAIT) && BSG_LA_WAIT) || (defined(BSG_ONLY_LA) && BSG_ONLY_LA)
  return 0;                          // (the lookahead's debug builds test the lookahead alone)
#else
  if (c->cfg.env_kind != BSG_ENV_MERGE || c->cfg.autoreset_mode != BSG_AUTORESET_NEXT_STEP ||
      c->cfg.max_episode_steps < 1 || c->cfg.max_episode_steps > bsg::TJ_SMAX)
    return 0;
  return (int64_t)(8 * bsg::tj_doubles((size_t)c->cfg.num_envs, (size_t)c->cfg.num_ac,
                                       (size_t)c->cfg.max_episode_steps));
#endif
}

int32_t bsg_set_trajectory(bsg_ctx* c, void* scratch, int64_t bytes, int32_t flags) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_set_trajectory: null ctx");
  if (int r = traj_quiesce(c)) return r;
  if (!scratch) {
    c->traj = nullptr;
    return BSG_OK;
  }
  const int64_t need = bsg_trajectory_bytes(c);
  if (need <= 0)
    return fail(BSG_E_UNSUPPORTED, "bsg_set_trajectory: MergeEnv with NEXT_STEP autoreset and a "
                "TimeLimit of 1..%d steps only", bsg::TJ_SMAX);
  if (!c->la) return fail(BSG_E_STATE, "bsg_set_trajectory: bind the lookahead scratch first");
  if (bytes < need)
    return fail(BSG_E_INVALID_ARG, "bsg_set_trajectory: scratch too small (need %lld bytes)",
                (long long)need);
  if (reinterpret_cast<uintptr_t>(scratch) & 7)
    return fail(BSG_E_INVALID_ARG, "bsg_set_trajectory: scratch must be 8-byte aligned");
  if (flags & ~BSG_TRAJ_SYNC) return fail(BSG_E_INVALID_ARG, "bsg_set_trajectory: unknown flags");
  hipError_t e = hipSetDevice(c->cfg.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  if (!c->prod_st) {
    int least = 0, greatest = 0;
    e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    // BSG_TRAJ_QPRIO=normal (A/B runs): the producer stream at the default priority
    const char* qp = std::getenv("BSG_TRAJ_QPRIO");
    const int prio = (qp && std::strcmp(qp, "normal") == 0) ? 0 : least;
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->prod_st, hipStreamNonBlocking, prio);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_step, hipEventDisableTiming);
    for (int k = 0; k < 4 && e == hipSuccess; ++k)
      e = hipEventCreateWithFlags(&c->ev_prod[k], hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(e, "bsg_set_trajectory: stream / events");
  }
  // headers of no generation (0xFF..), counters zero; entries are written before use
  const size_t head = 8 * (size_t)c->cfg.num_envs * (1 + bsg::TJ_P);
  e = hipMemset(scratch, 0xFF, head);
  if (e == hipSuccess) e = hipMemset(scratch, 0, 8 * (size_t)c->cfg.num_envs);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "bsg_set_trajectory: hipMemset");
  c->traj = static_cast<double*>(scratch);
  c->traj_sync = (flags & BSG_TRAJ_SYNC) != 0;
  if (const char* na = std::getenv("BSG_TRAJ_NOASYNC")) c->traj_noasync = std::atoi(na) != 0;
  if (const char* wp = std::getenv("BSG_TRAJ_WPRIO")) c->traj_wprio = std::atoi(wp);
  if (const char* ev = std::getenv("BSG_TRAJ_EVERY")) c->traj_every = std::max(1, std::atoi(ev));
  if (const char* sl = std::getenv("BSG_TRAJ_SLEEP")) c->traj_sleep = std::max(0, std::atoi(sl));
  traj_new_gen(c);
  c->steps_since_prod = 1 << 20;
  return BSG_OK;
}

int32_t bsg_trajectory_info(const bsg_ctx* c, int64_t* out /* [4] */) {
  if (!c || !out) return fail(BSG_E_INVALID_ARG, "bsg_trajectory_info: null argument");
  out[0] = c->traj ? 1 : 0;
  out[1] = c->prod_launches;
  out[2] = (int64_t)c->prod_out;
  out[3] = (int64_t)c->traj_gen;
  return BSG_OK;
}

int32_t bsg_set_learner(bsg_ctx* c, float* learner) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_set_learner: null ctx");
  if (!c->bound) return fail(BSG_E_STATE, "bsg_set_learner: buffers not bound");
  c->bufs.learner = learner;
  return BSG_OK;
}

int32_t bsg_reset(bsg_ctx* c, const uint8_t* env_mask, const double* spawn, void* stream) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_reset: null ctx");
  if (!c->bound) return fail(BSG_E_STATE, "bsg_reset: buffers not bound");
  return launch(c, bsg::MODE_RESET, nullptr, spawn, env_mask, stream);
}

int32_t bsg_step(bsg_ctx* c, const double* actions, const double* spawn, void* stream) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_step: null ctx");
  if (!c->bound) return fail(BSG_E_STATE, "bsg_step: buffers not bound");
  if (!actions) return fail(BSG_E_INVALID_ARG, "bsg_step: actions is NULL");
  return launch(c, bsg::MODE_STEP, actions, spawn, nullptr, stream);
}

int32_t bsg_step_gather(bsg_ctx* c, bsg_comm* comm, const double* actions, const double* spawn,
                        float* rows, float* gathered, int32_t slot, void* stream) {
  if (!c || !comm) return fail(BSG_E_INVALID_ARG, "bsg_step_gather: null ctx/comm");
  if (!c->bound) return fail(BSG_E_STATE, "bsg_step_gather: buffers not bound");
  if (!actions || !rows || !gathered) return fail(BSG_E_INVALID_ARG, "bsg_step_gather: null buffer");
  // rows[slot] was last read by the gather of BSG_COMM_SLOTS steps ago (a ring): the step
  // writes it after that gather (usually known complete already: no stream wait)
  if (bsg_comm_wait(comm, slot, stream) != BSG_OK)
    return fail(BSG_E_HIP, "bsg_step_gather: %s", bsg_comm_last_error());
  c->bufs.learner = rows;
  if (int r = launch(c, bsg::MODE_STEP, actions, spawn, nullptr, stream)) return r;
  const int64_t count = (int64_t)c->cfg.num_envs * (c->obs_dim + 3);
  if (bsg_comm_all_gather(comm, rows, gathered, count, slot, stream) != BSG_OK)
    return fail(BSG_E_HIP, "bsg_step_gather: %s", bsg_comm_last_error());
  return BSG_OK;
}

int32_t bsg_set_wind(bsg_ctx* c, const bsg_wind* w) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_set_wind: null ctx");
  const int base = bsg_obs_dim(c->cfg.env_kind, c->cfg.num_ac, c->cfg.num_ac_state);
  bsg::WindDev d{};
  if (w && w->num_points > 0) {
    if (w->num_points > 4096)
      return fail(BSG_E_INVALID_ARG, "bsg_set_wind: num_points must be <= 4096 (got %lld)", (long long)(w->num_points));
    if (w->num_levels != 1 && w->num_levels != BSG_WIND_NALT)
      return fail(BSG_E_INVALID_ARG, "bsg_set_wind: num_levels must be 1 or BSG_WIND_NALT (got %lld)", (long long)(w->num_levels));
    if (!w->lat || !w->lon || !w->vnorth || !w->veast)
      return fail(BSG_E_INVALID_ARG, "bsg_set_wind: null table pointer");
    d.np = w->num_points;
    d.nlev = w->num_levels;
    d.dim = d.nlev > 1 ? 3 : (d.np == 1 ? 1 : 2);
    d.augment = w->augment_obs != 0;
    d.lat = w->lat; d.lon = w->lon; d.vn = w->vnorth; d.ve = w->veast;
  }
  c->wind = d;
  c->obs_dim = base + (d.augment ? 2 : 0);
  c->bound = false;
  c->la_dirty = true;
  return BSG_OK;
}

int32_t bsg_ctx_obs_dim(const bsg_ctx* c) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_ctx_obs_dim: null ctx");
  return c->obs_dim;
}

int32_t bsg_policy_sac(const bsg_sac_actor* w, const float* obs, int32_t num_envs,
                       int32_t obs_stride, const float* eps, double* actions, float* log_prob,
                       void* stream) {
  if (!w) return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: null actor");
  if (num_envs > 0 && (!obs || !actions)) return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: null obs/actions");
  if (w->hidden != 256)
    return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: hidden must be 256 (got %lld)", (long long)(w->hidden));
  if (w->obs_dim < 1 || w->obs_dim > 256)
    return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: obs_dim must be in [1, 256] (got %lld)", (long long)(w->obs_dim));
  if (w->act_dim < 1 || w->act_dim > 4)
    return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: act_dim must be in [1, 4] (got %lld)", (long long)(w->act_dim));
  if (num_envs < 0) return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: num_envs < 0");
  if (obs_stride < w->obs_dim)
    return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: obs_stride < obs_dim (%lld)", (long long)(obs_stride));
  if (!w->w0 || !w->b0 || !w->w1 || !w->b1 || !w->w_mu || !w->b_mu || !w->w_ls || !w->b_ls)
    return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: null weight pointer");
  if (reinterpret_cast<uintptr_t>(w->w1) & 15)
    return fail(BSG_E_INVALID_ARG, "bsg_policy_sac: w1 must be 16-byte aligned");
  if (num_envs == 0) return BSG_OK;
  hipError_t e = bsg::launch_sac_actor(*w, obs, num_envs, obs_stride, eps, actions, log_prob,
                                       static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "bsg_policy_sac launch");
  return BSG_OK;
}

int32_t bsg_set_stamps(bsg_ctx* c, void* buf) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_set_stamps: null ctx");
#if defined(BSG_STAMPS) && BSG_STAMPS
  c->stamps = static_cast<unsigned long long*>(buf);
  return BSG_OK;
#else
  (void)buf;
  return fail(BSG_E_UNSUPPORTED, "bsg_set_stamps: library built without -DBSG_STAMPS=1");
#endif
}

int32_t bsg_set_timing(bsg_ctx* c, int32_t enable) {
  if (!c) return fail(BSG_E_INVALID_ARG, "bsg_set_timing: null ctx");
  if (enable < 0) return fail(BSG_E_INVALID_ARG, "bsg_set_timing: negative interval");
  c->timing = enable;
  c->launch_count = 0;
  return BSG_OK;
}

int32_t bsg_step_timing(bsg_ctx* c, double* total_ms, int32_t* launches) {
  if (!c || !total_ms || !launches) return fail(BSG_E_INVALID_ARG, "bsg_step_timing: null argument");
  // fold every pending pair; on a failure the pairs folded so far stay in the totals
  // (reported by the next call) and only the unfolded ones remain pending
  for (size_t i = 0; i < c->pending.size(); ++i) {
    if (int r = fold_pair(c, c->pending[i])) {
      c->pending.erase(c->pending.begin(), c->pending.begin() + i);
      return r;
    }
  }
  c->pending.clear();
  *total_ms = c->folded_ms;
  *launches = c->folded_n;
  c->folded_ms = 0.0;
  c->folded_n = 0;
  return BSG_OK;
}

}  // extern "C"
