"""ctypes binding of libbsg.so (include/bsg.h).

The product path: every env step of ``bluesky_gym`` goes through these entry points.
There is no CPU fallback -- if the HIP library is missing or no HIP device is present,
construction raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BSG_LIBRARY", os.path.join(_HERE, "_lib", "libbsg.so"))

ABI_VERSION = 2
MAX_ROUTE = 4
WIND_NALT = 451

ENV_MERGE, ENV_VERTICAL_CR, ENV_DESCENT, ENV_HORIZONTAL_CR = 0, 1, 2, 3
ENV_STATIC_OBSTACLE, ENV_SECTOR_CR, ENV_PLAN_WAYPOINT = 4, 5, 6
FLAG_RESET_PENDING, FLAG_AC_PRESENT, FLAG_SPAWN_OVERFLOW = 1, 2, 4   # include/bsg.h BSG_FLAG_*
AUTORESET_NONE, AUTORESET_NEXT_STEP, AUTORESET_SAME_STEP = 0, 1, 2

E_CODES = {-1: "BSG_E_INVALID_ARG", -2: "BSG_E_HIP", -3: "BSG_E_STATE", -4: "BSG_E_UNSUPPORTED"}

_dp = C.POINTER(C.c_double)
_fp = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)


class BsgConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("env_kind", C.c_int32),
        ("num_envs", C.c_int32),
        ("num_ac", C.c_int32),
        ("num_ac_state", C.c_int32),
        ("action_frequency", C.c_int32),
        ("simdt", C.c_double),
        ("max_episode_steps", C.c_int32),
        ("autoreset_mode", C.c_int32),
        ("compute_cd", C.c_int32),
        ("device", C.c_int32),
        ("seed", C.c_uint64),
        ("route_len", C.c_int32),
        ("env_offset", C.c_int32),
        ("kind_option", C.c_int32),
        ("reserved0", C.c_int32),
        ("route_lat", C.c_double * MAX_ROUTE),
        ("route_lon", C.c_double * MAX_ROUTE),
        ("route_next_qdr", C.c_double * MAX_ROUTE),
        ("wpt_lat", C.c_double * 2),
        ("wpt_lon", C.c_double * 2),
    ]


# (name, ctype pointer) in include/bsg.h order
BUFFER_FIELDS = [
    ("lat", _dp), ("lon", _dp), ("alt", _dp), ("hdg", _dp), ("tas", _dp), ("cas", _dp),
    ("vs", _dp), ("ax", _dp), ("ap_trk", _dp), ("selspd", _dp), ("selalt", _dp),
    ("selvs", _dp), ("nav", _i32p), ("gs", _dp), ("trk", _dp), ("memo_cache", _dp),
    ("step_count", _i32p), ("flags", _i32p), ("episode", _u32p), ("wpt_reach", _i32p),
    ("faf_reached", _i32p), ("total_intrusions", _i32p), ("total_reward", _dp),
    ("drift_sum", _dp), ("target_alt", _dp), ("final_altitude", _dp),
    ("env_wpt_lat", _dp), ("env_wpt_lon", _dp), ("env_geom", _dp), ("env_aux", _dp),
    ("obs", _fp), ("final_obs", _fp), ("reward", _fp), ("terminated", _u8p),
    ("truncated", _u8p), ("topk", _i32p), ("intr_mask", _u64p), ("conf_mask", _u64p),
    ("los_mask", _u64p), ("tcpamax", _fp), ("min_sep", _fp), ("ep_info", _dp),
    ("learner", _fp),
]


class BsgBuffers(C.Structure):
    _fields_ = [(n, t) for n, t in BUFFER_FIELDS]


class BsgWind(C.Structure):
    _fields_ = [
        ("num_points", C.c_int32),
        ("num_levels", C.c_int32),
        ("augment_obs", C.c_int32),
        ("reserved", C.c_int32),
        ("lat", _dp), ("lon", _dp), ("vnorth", _dp), ("veast", _dp),
    ]


EXPORTED_SYMBOLS = (
    "bsg_abi_version", "bsg_last_error", "bsg_obs_dim", "bsg_action_dim", "bsg_spawn_width",
    "bsg_create", "bsg_destroy", "bsg_bind", "bsg_reset", "bsg_step", "bsg_set_timing",
    "bsg_step_timing", "bsg_set_stamps", "bsg_set_wind", "bsg_ctx_obs_dim", "bsg_geom_width",
    "bsg_set_learner", "bsg_policy_sac", "bsg_lookahead_bytes", "bsg_set_lookahead",
    "bsg_comm_last_error", "bsg_comm_unique_id", "bsg_comm_create", "bsg_comm_destroy",
    "bsg_comm_all_gather", "bsg_comm_wait", "bsg_comm_get_info", "bsg_step_gather",
    "bsg_comm_all_reduce", "bsg_set_params", "bsg_trajectory_bytes", "bsg_set_trajectory",
    "bsg_trajectory_info",
)
TRAJ_SYNC = 1                # include/bsg.h BSG_TRAJ_SYNC
# include/bsg.h BSG_MP_*: MergeEnv-v0's module constants (merge_env.py:13-46), in this order,
# with the reference's values (bsg_create's defaults)
MERGE_PARAMS = (("D_HEADING", 15.0), ("D_SPEED", 20.0), ("INTRUSION_DISTANCE", 4.0),
                ("DISTANCE_MARGIN", 10.0), ("REACH_REWARD", 1.0), ("DRIFT_PENALTY", -0.1),
                ("INTRUSION_PENALTY", -1.0), ("SPAWN_DISTANCE_MIN", 50.0),
                ("SPAWN_DISTANCE_MAX", 200.0), ("INTRUDER_DISTANCE_MIN", 20.0),
                ("INTRUDER_DISTANCE_MAX", 500.0))
REDUCE_SUM, REDUCE_AVG = 0, 1   # include/bsg.h BSG_REDUCE_*
COMM_ID_BYTES = 128          # include/bsg.h BSG_COMM_ID_BYTES
COMM_SLOTS = 16              # BSG_COMM_SLOTS


class BsgCommInfo(C.Structure):
    """include/bsg.h bsg_comm_info."""
    _fields_ = [("nranks", C.c_int32), ("rank", C.c_int32), ("device", C.c_int32),
                ("use_graphs", C.c_int32), ("gathers", C.c_int64), ("graph_hits", C.c_int64),
                ("graph_captures", C.c_int64), ("reduces", C.c_int64)]


class BsgSacActor(C.Structure):
    """include/bsg.h bsg_sac_actor: device pointers of an SB3 SAC actor's weights."""
    _fields_ = [("obs_dim", C.c_int32), ("act_dim", C.c_int32), ("hidden", C.c_int32),
                ("reserved", C.c_int32)] + [(n, C.c_void_p) for n in (
                    "w0", "b0", "w1", "b1", "w_mu", "b_mu", "w_ls", "b_ls")]

_lib = None


class BsgError(RuntimeError):
    pass


def load_library(path: str | None = None):
    """Load libbsg.so once and declare every signature of include/bsg.h."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise BsgError(f"libbsg.so not found at {p}: build it with "
                       f"`python -c 'import __graft_entry__ as g; g.build()'` or `make -C "
                       f"bluesky-gym-hallucination_amd/csrc`")
    lib = C.CDLL(p)
    lib.bsg_abi_version.restype = C.c_int32
    lib.bsg_abi_version.argtypes = []
    lib.bsg_last_error.restype = C.c_char_p
    lib.bsg_last_error.argtypes = []
    for fn in ("bsg_obs_dim",):
        getattr(lib, fn).restype = C.c_int32
        getattr(lib, fn).argtypes = [C.c_int32, C.c_int32, C.c_int32]
    lib.bsg_action_dim.restype = C.c_int32
    lib.bsg_action_dim.argtypes = [C.c_int32]
    lib.bsg_spawn_width.restype = C.c_int32
    lib.bsg_spawn_width.argtypes = [C.c_int32, C.c_int32]
    lib.bsg_geom_width.restype = C.c_int32
    lib.bsg_geom_width.argtypes = [C.c_int32, C.c_int32]
    lib.bsg_create.restype = C.c_int32
    lib.bsg_create.argtypes = [C.POINTER(BsgConfig), C.POINTER(C.c_void_p)]
    lib.bsg_destroy.restype = C.c_int32
    lib.bsg_destroy.argtypes = [C.c_void_p]
    lib.bsg_bind.restype = C.c_int32
    lib.bsg_bind.argtypes = [C.c_void_p, C.POINTER(BsgBuffers)]
    lib.bsg_set_learner.restype = C.c_int32
    lib.bsg_set_learner.argtypes = [C.c_void_p, C.c_void_p]
    lib.bsg_reset.restype = C.c_int32
    lib.bsg_reset.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.bsg_step.restype = C.c_int32
    lib.bsg_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.bsg_set_timing.restype = C.c_int32
    lib.bsg_set_timing.argtypes = [C.c_void_p, C.c_int32]
    lib.bsg_step_timing.restype = C.c_int32
    lib.bsg_step_timing.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32)]
    lib.bsg_set_stamps.restype = C.c_int32
    lib.bsg_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
    lib.bsg_set_wind.restype = C.c_int32
    lib.bsg_set_wind.argtypes = [C.c_void_p, C.POINTER(BsgWind)]
    lib.bsg_ctx_obs_dim.restype = C.c_int32
    lib.bsg_ctx_obs_dim.argtypes = [C.c_void_p]
    lib.bsg_lookahead_bytes.restype = C.c_int64
    lib.bsg_lookahead_bytes.argtypes = [C.c_void_p]
    lib.bsg_trajectory_bytes.restype = C.c_int64
    lib.bsg_trajectory_bytes.argtypes = [C.c_void_p]
    lib.bsg_set_trajectory.restype = C.c_int32
    lib.bsg_set_trajectory.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]
    lib.bsg_trajectory_info.restype = C.c_int32
    lib.bsg_trajectory_info.argtypes = [C.c_void_p, C.c_void_p]
    lib.bsg_set_lookahead.restype = C.c_int32
    lib.bsg_set_lookahead.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    lib.bsg_policy_sac.restype = C.c_int32
    lib.bsg_policy_sac.argtypes = [C.POINTER(BsgSacActor), C.c_void_p, C.c_int32, C.c_int32,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.bsg_comm_last_error.restype = C.c_char_p
    lib.bsg_comm_last_error.argtypes = []
    lib.bsg_comm_unique_id.restype = C.c_int32
    lib.bsg_comm_unique_id.argtypes = [C.c_void_p]
    lib.bsg_comm_create.restype = C.c_int32
    lib.bsg_comm_create.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
    lib.bsg_comm_destroy.restype = C.c_int32
    lib.bsg_comm_destroy.argtypes = [C.c_void_p]
    lib.bsg_comm_all_gather.restype = C.c_int32
    lib.bsg_comm_all_gather.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32,
                                        C.c_void_p]
    lib.bsg_comm_wait.restype = C.c_int32
    lib.bsg_comm_wait.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
    lib.bsg_set_params.restype = C.c_int32
    lib.bsg_set_params.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    lib.bsg_comm_all_reduce.restype = C.c_int32
    lib.bsg_comm_all_reduce.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]
    lib.bsg_comm_get_info.restype = C.c_int32
    lib.bsg_comm_get_info.argtypes = [C.c_void_p, C.POINTER(BsgCommInfo)]
    lib.bsg_step_gather.restype = C.c_int32
    lib.bsg_step_gather.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_int32, C.c_void_p]
    if lib.bsg_abi_version() != ABI_VERSION:
        raise BsgError(f"libbsg ABI {lib.bsg_abi_version()} != expected {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        lib = load_library()
        msg = lib.bsg_last_error().decode(errors="replace")
        raise BsgError(f"{what} failed ({E_CODES.get(rc, rc)}): {msg}")


def check_comm(rc: int, what: str):
    """Like check() for the bsg_comm_* calls (their own error string)."""
    if rc != 0:
        msg = load_library().bsg_comm_last_error().decode(errors="replace")
        raise BsgError(f"{what} failed ({rc}): {msg}")
