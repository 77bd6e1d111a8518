// bsg_dispatch.cpp -- launch_step: the env kind picks its translation unit's launcher.
#include "bsg_internal.h"

namespace bsg {

static_assert(BSG_ENV_MERGE == 0 && BSG_ENV_VERTICAL_CR == 1 && BSG_ENV_DESCENT == 2 &&
                  BSG_ENV_HORIZONTAL_CR == 3 && BSG_ENV_STATIC_OBSTACLE == 4 &&
                  BSG_ENV_SECTOR_CR == 5 && BSG_ENV_PLAN_WAYPOINT == 6,
              "launch_kind_<n> suffixes are the BSG_ENV_* values");

hipError_t launch_step(const KParams& p, hipStream_t st) {
#if defined(BSG_ONLY_MERGE) && BSG_ONLY_MERGE
  // experiment builds (tools/flag_sweep.sh, tools/variants.sh): Merge only, for fast sweeps
  return p.cfg.env_kind == BSG_ENV_MERGE ? launch_kind_0(p, st) : hipErrorInvalidValue;
#elif defined(BSG_ONLY_LA) && BSG_ONLY_LA
  // lookahead debug builds (Makefile la-debug): the two kinds with a lookahead
  switch (p.cfg.env_kind) {
    case BSG_ENV_MERGE: return launch_kind_0(p, st);
    case BSG_ENV_VERTICAL_CR: return launch_kind_1(p, st);
    default: return hipErrorInvalidValue;
  }
#else
  switch (p.cfg.env_kind) {
    case BSG_ENV_MERGE: return launch_kind_0(p, st);
    case BSG_ENV_VERTICAL_CR: return launch_kind_1(p, st);
    case BSG_ENV_DESCENT: return launch_kind_2(p, st);
    case BSG_ENV_HORIZONTAL_CR: return launch_kind_3(p, st);
    case BSG_ENV_STATIC_OBSTACLE: return launch_kind_4(p, st);
    case BSG_ENV_SECTOR_CR: return launch_kind_5(p, st);
    case BSG_ENV_PLAN_WAYPOINT: return launch_kind_6(p, st);
    default: return hipErrorInvalidValue;
  }
#endif
}

}  // namespace bsg
