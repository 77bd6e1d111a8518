// bsg_internal.h -- launch parameters shared by the C ABI (bsg_abi.cpp) and the kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/bsg.h"

namespace bsg {

using Buffers = bsg_buffers;

enum { MODE_STEP = 0, MODE_RESET = 1 };

struct Route {
  int len;
  double lat[BSG_MAX_ROUTE], lon[BSG_MAX_ROUTE], next_qdr[BSG_MAX_ROUTE];
  double rwgs[BSG_MAX_ROUTE];   // WGS84 radius rwgs84(lat) of each waypoint (host libm; used
                                // only inside rounding-slack bounds, bsg_device.h)
};

struct WindDev {
  int np;                    // points (0: wind off)
  int nlev;                  // 1 or BSG_WIND_NALT
  int dim;                   // 1 constant, 2 horizontal IDW, 3 IDW + altitude levels
  int augment;               // obs carries wind_u / wind_v
  const double *lat, *lon, *vn, *ve;
};

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
};

hipError_t launch_step(const KParams& p, hipStream_t stream);

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
