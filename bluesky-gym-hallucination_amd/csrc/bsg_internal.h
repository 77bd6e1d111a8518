// bsg_internal.h -- launch parameters shared by the C ABI (bsg_abi.cpp) and the kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/bsg.h"

namespace bsg {

using Buffers = bsg_buffers;

// MODE_PRIME: the lookahead's priming pass (bsg_abi.cpp launch), lookahead workgroups only
enum { MODE_STEP = 0, MODE_RESET = 1, MODE_PRIME = 2 };

struct Route {
  int len;
  double lat[BSG_MAX_ROUTE], lon[BSG_MAX_ROUTE], next_qdr[BSG_MAX_ROUTE];
  double rwgs[BSG_MAX_ROUTE];   // WGS84 radius rwgs84(lat) of each waypoint (host libm; used
                                // only inside rounding-slack bounds, bsg_device.h)
};

// The per-waypoint terms of the LNAV loop, computed once on the host with the device's own
// functions (bit-identical there, tools/probe/fastmath_probe.hip): sincos_t of lat * D2R,
// lon * D2R, pymod360(next_qdr).  At the end of KParams, so that the offsets of the fields
// every launch reads stay as they were (moving the buffer pointers measured +2 % on
// Vertical / Descent).
struct RouteTrig {
  double sinlat[BSG_MAX_ROUTE], coslat[BSG_MAX_ROUTE], lonr[BSG_MAX_ROUTE], pnq[BSG_MAX_ROUTE];
};

struct WindDev {
  int np;                    // points (0: wind off)
  int nlev;                  // 1 or BSG_WIND_NALT
  int dim;                   // 1 constant, 2 horizontal IDW, 3 IDW + altitude levels
  int augment;               // obs carries wind_u / wind_v
  const double *lat, *lon, *vn, *ve;
};

// Lookahead scratch layout (bsg_set_lookahead; bsg_kernels.hip lookahead_role), in doubles
// for EN = E*N: two slots of LA_F fields x EN (LA_STATE state fields, then -- Vertical, la_cd
// -- the intruder pairs' StateBased rows as u64 bits: conflict row, LoS row, tcpamax), the
// lookahead blocks' memo [LA_MC][EN], two tag rows [E] (u64), two rows [E] of the intruder
// pairs' minimum separation (bits of a double), then the env-scalar snapshot the lookahead
// waves read instead of the live env scalars: [2 launch parities][E][2] u64 (bsg_kernels.hip
// la_snap).  Debug builds with -DBSG_LA_WAIT=1 append [E] u64 phase-A flags (tests only).
// Last, Merge's spawn cache (bsg_kernels.hip spawn_cache_*): [3][EN] the next episode's
// creation lat / lon / heading per aircraft, then [E] u64 the episode each env's entries
// were drawn for.
constexpr int LA_STATE = 10;
constexpr int LA_F = LA_STATE + 3;
constexpr int LA_MC = 2;           // = MC_FIELDS (bsg_kernels.hip)
#if defined(BSG_LA_WAIT) && BSG_LA_WAIT
constexpr size_t LA_WAIT_E = 1;
#else
constexpr size_t LA_WAIT_E = 0;
#endif
__host__ __device__ constexpr size_t la_doubles(size_t E, size_t N) {
  return (2 * LA_F + LA_MC) * E * N + (8 + LA_WAIT_E) * E + 3 * E * N + E;
}
__host__ __device__ constexpr size_t la_sc_offset(size_t E, size_t N) {
  return (2 * LA_F + LA_MC) * E * N + (8 + LA_WAIT_E) * E;
}

// Trajectory store (bsg_set_trajectory; MergeEnv with the lookahead, NEXT_STEP autoreset, a
// TimeLimit of S <= TJ_SMAX steps).  A Merge intruder's whole episode is a function of (seed,
// env, Philox episode counter) alone (merge_env.py:148-158, RESO OFF), so produce_kernel flies
// future episodes ahead on a low-priority stream -- every post-step state of steps 1..S and
// the intruder pairs' StateBased rows -- and the step kernel's lookahead waves copy the next
// step's entry into the lookahead slot instead of running ten substeps on the launch's
// critical path.  A producer wave releases each step as it stores it (the header counts the
// steps held), so an episode is usable step by step while it is being flown; a later launch
// resumes an episode from its last stored step.
// Layout, in doubles: [E] u64 copy counters (diagnostics), [E][TJ_P] u64 headers (tj_pack:
// generation | steps held | episode counter), entries [TJ_P][S][TJ_F][EN] (the lookahead
// slot's LA_F fields and the env's minimum separation over the intruder pairs at the
// ownship's index), then the producers' memo [TJ_D + 1][LA_MC][EN].  Slot = episode counter
// % TJ_P.
constexpr int TJ_P = 4;
constexpr int TJ_F = LA_F + 1;
constexpr int TJ_D = 3;            // a producer launch covers the episodes 1..TJ_D ahead
constexpr int TJ_SMAX = 63;        // (6 bits of the header)
__host__ __device__ constexpr size_t tj_doubles(size_t E, size_t N, size_t S) {
  return E + TJ_P * E + TJ_P * S * TJ_F * E * N + (TJ_D + 1) * LA_MC * E * N;
}

// Passed by value to every launch (kernarg segment).
struct KParams {
  bsg_config cfg;
  Route route;
  Buffers b;
  int mode;
  int E, N, K, obs_dim, spawn_width;
  uint64_t seed;
  const double* actions;     // [E, A]
  const double* spawn;       // [E, spawn_width] or nullptr (Philox)
  const uint8_t* env_mask;   // [E] or nullptr (all)  -- reset mode only
  unsigned long long* stamps; // diagnostics (BSG_STAMPS builds only)
  unsigned lds_pad;          // extra dynamic LDS per workgroup (occupancy shaping)
  WindDev wind;
  int wpos;                  // obs offset of wind_u (sorted-key position) when augmenting
  // lookahead (bsg_set_lookahead; Merge, no wind, not SAME_STEP): workgroups
  // [la_grid0, 2*la_grid0) propagate the intruders one RL step ahead into `la`
  double* la;                // scratch (layout: bsg_kernels.hip la_*), nullptr = off
  int la_par;                // slot the main workgroups read (a step's lookahead writes 1 - la_par)
  uint32_t la_gen;           // generation: tags of other generations are stale
  int la_grid0;              // main workgroups (set by the launcher)
  int no_fastpath;           // BSG_NO_FASTPATH=1 at bsg_create: the general substep only
                             // (tests compare the specialised paths against it)
  RouteTrig route_t;         // (last: see RouteTrig)
  int prio_sw_num, prio_sw_den;  // substep priority switch point (set by the launcher)
  int la_cd;                 // the lookahead waves also run the intruder pairs' StateBased CD
                             // (set by the launcher: VerticalCREnv with compute_cd)
  uint32_t la_seq;           // launches since the lookahead scratch was (re)armed: its parity
                             // picks the env-scalar snapshot a launch reads (the main waves
                             // write the other one for the next launch)
  // Merge: the creation state every aircraft of every env spawns with (same CAS, same
  // altitude; bsg_abi.cpp computes it once with the kernels' own functions,
  // spawn_consts_merge): [0] tas, [1] cas of Traffic.cre, [2] the speed memo's ap_tas,
  // [3] its allow_tas entry (> 0: the 'level' form, bsg_kernels.hip Memo).  spawn_k_ok = 0:
  // not available (cre and the memo as before).
  double spawn_k[8];
  int spawn_k_ok;
  // the env module's constants (bsg_set_params, include/bsg.h BSG_MP_*; Merge)
  double kp[BSG_MERGE_NPARAMS];
  // trajectory store (bsg_set_trajectory; tj_doubles): nullptr = off
  double* traj;
  uint32_t traj_gen;         // generation: headers of other generations are stale
  int traj_S;                // steps per stored episode (the TimeLimit)
  int prod_d0, prod_d1;      // produce_kernel: episodes ahead of the running one it covers
  int prod_q;                // produce_kernel: steps per episode this launch flies (at most)
  int prod_sleep;            // produce_kernel: s_sleep(127) rounds after each step of an
                             // episode >= 2 ahead (duty-cycle throttle; BSG_TRAJ_SLEEP)
  int prod_async;            // produce_kernel: a step's producer launch, which continues the
                             // running episode only (0: a reset's, which flies it from its
                             // creation)
  int is_prod;               // produce_kernel: its waves run at the lowest priority
};

hipError_t launch_step(const KParams& p, hipStream_t stream);

// produce_kernel (Merge translation unit): the episodes prod_d0..prod_d1 ahead of each env's
// running one into the trajectory store, on `stream`
// the lookahead-free Merge launch (its own translation unit: bsg_kernels.hip BSG_MERGE_NL_TU)
hipError_t launch_merge_nl(const KParams& p, int gs, int grid, hipStream_t st);
hipError_t launch_produce(const KParams& p, hipStream_t stream);

// Merge's creation-state constants (KParams::spawn_k) into out[0..7] (device; out[4] = 1.0
// when valid; out[5..7] the creation altitude's atmosphere), one thread, on `stream` (bsg_kernels.hip, the Merge translation unit)
hipError_t spawn_consts_merge(double spd, double alt, double* out, hipStream_t stream);

// per-kind launchers, one translation unit each (bsg_kernels.hip -DBSG_KIND_TU=<kind>;
// the suffix is the BSG_ENV_* value)
hipError_t launch_kind_0(const KParams& p, hipStream_t stream);
hipError_t launch_kind_1(const KParams& p, hipStream_t stream);
hipError_t launch_kind_2(const KParams& p, hipStream_t stream);
hipError_t launch_kind_3(const KParams& p, hipStream_t stream);
hipError_t launch_kind_4(const KParams& p, hipStream_t stream);
hipError_t launch_kind_5(const KParams& p, hipStream_t stream);
hipError_t launch_kind_6(const KParams& p, hipStream_t stream);

// the fused SAC actor (bsg_policy.hip)
hipError_t launch_sac_actor(const bsg_sac_actor& w, const float* obs, int E, int ostride,
                            const float* eps, double* act, float* logp, hipStream_t stream);

}  // namespace bsg
