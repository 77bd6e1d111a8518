/*
 * bsg.h -- C ABI of libbsg.so, the MI355X-native vectorised BlueSky-Gym step path.
 *
 * Drop-in boundary: the reference exposes one Gymnasium env per process
 * (bluesky_gym/envs/merge_env.py:48, vertical_cr_env.py:47, descent_env.py:32) whose
 * reset()/step() drive a process-global BlueSky singleton.  This library replaces that
 * pair with a device-resident structure-of-arrays batch of E envs, stepped by one HIP
 * launch per RL step.  The Python host mirror (bluesky_gym/_native.py, ctypes) binds
 * exactly these symbols; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Caller owns ALL memory.  Every pointer in bsg_buffers is a device pointer
 *     (hipMalloc / torch.cuda tensor).  The library stores them non-owning.
 *   - All launches are asynchronous on the caller's stream (hipStream_t passed as void*);
 *     no call synchronises the device.
 *   - Return 0 on success, a negative BSG_E_* code otherwise; bsg_last_error() gives the
 *     thread-local message.  No C++ exception crosses the ABI.
 *   - Aircraft arrays are [num_envs][num_ac] row-major (env-major); aircraft 0 of each
 *     env is the ownship ('KL001'), 1..num_ac-1 the intruders ('INT{i}' / creconfs).
 */
#ifndef BSG_H_
#define BSG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSG_ABI_VERSION 2
#define BSG_MAX_AC 64          /* aircraft per env (one wavefront) */
#define BSG_MAX_ROUTE 4
#define BSG_WIND_NALT 451      /* wind profile levels: 0..45000 ft every 100 ft */

enum {
  BSG_OK = 0,
  BSG_E_INVALID_ARG = -1,
  BSG_E_HIP = -2,
  BSG_E_STATE = -3,
  BSG_E_UNSUPPORTED = -4
};

enum { BSG_ENV_MERGE = 0, BSG_ENV_VERTICAL_CR = 1, BSG_ENV_DESCENT = 2,
       BSG_ENV_HORIZONTAL_CR = 3, BSG_ENV_STATIC_OBSTACLE = 4, BSG_ENV_SECTOR_CR = 5,
       BSG_ENV_PLAN_WAYPOINT = 6 };

/* bsg_buffers.flags bits */
enum { BSG_FLAG_RESET_PENDING = 1,   /* NEXT_STEP autoreset due on the next step */
       BSG_FLAG_AC_PRESENT = 2,      /* Descent / PlanWaypoint: KL001 exists.  Their reset()
                                        does not clear the traffic, so a reset after a
                                        truncation keeps the aircraft (cre refused,
                                        descent_env.py:173, plan_waypoint_env.py:164); the
                                        terminal step deletes it (:201-204, :189-193) */
       BSG_FLAG_SPAWN_OVERFLOW = 4 };/* SectorCR: this episode drew more aircraft than the
                                        capacity N (sector_cr_env.py:95-100 has no cap); the
                                        device spawned N of them.  The Python layer raises
                                        on it, as the host-spawn path does */

/* Vector-env autoreset conventions:
 *   NEXT_STEP: Gymnasium >= 1.0 VectorEnv default -- the step AFTER a done step resets
 *              the env (action ignored, reward 0, terminated/truncated false).
 *   SAME_STEP: SB3 VecEnv -- a done env is reset inside the same step; the terminal
 *              observation is written to final_obs, obs holds the reset observation. */
enum { BSG_AUTORESET_NONE = 0, BSG_AUTORESET_NEXT_STEP = 1, BSG_AUTORESET_SAME_STEP = 2 };

typedef struct bsg_config {
  int32_t abi_version;       /* = BSG_ABI_VERSION */
  int32_t env_kind;          /* BSG_ENV_* */
  int32_t num_envs;          /* E */
  int32_t num_ac;            /* N aircraft per env incl. ownship (merge_env.py:37 NUM_AC;
                                vertical: 1 + NUM_INTRUDERS, vertical_cr_env.py:45; descent: 1) */
  int32_t num_ac_state;      /* K nearest intruders in the Merge obs (merge_env.py:38) */
  int32_t action_frequency;  /* substeps per RL step (merge_env.py:35; vertical_cr_env.py:43) */
  double simdt;              /* s per substep ('DT 5' merge_env.py:86; 'DT 1' vertical_cr_env.py:95) */
  int32_t max_episode_steps; /* TimeLimit (bluesky_gym/__init__.py:9,27,45); 0 = none */
  int32_t autoreset_mode;    /* BSG_AUTORESET_* */
  int32_t compute_cd;        /* 1: StateBased all-pairs CPA outputs every step */
  int32_t device;            /* HIP device ordinal */
  uint64_t seed;             /* Philox key for device-side spawns */
  int32_t route_len;         /* Merge intruder route (ADDWPT FIX; DEST RWY, merge_env.py:155-156) */
  int32_t env_offset;        /* global id of env 0 of this batch (Philox counter); a shard of a
                                multi-GPU job passes its first global env id */
  int32_t kind_option;       /* SectorCR ac_density_mode: 0 "normal", 1 uniform
                                (sector_cr_env.py:45,95-100).  MergeEnv: the creation CAS of
                                every aircraft in m/s, 0 = the reference's AC_SPD = 100
                                (merge_env.py:30,119,154); a test hook for the log revision
                                of DESIGN.md §5.  0 for the other kinds */
  int32_t reserved0;
  double route_lat[BSG_MAX_ROUTE];
  double route_lon[BSG_MAX_ROUTE];
  double route_next_qdr[BSG_MAX_ROUTE]; /* qdrdist bearing wp k -> k+1; -999 for the last */
  double wpt_lat[2];         /* Merge drift targets: FIX, RWY (merge_env.py:98-101) */
  double wpt_lon[2];
} bsg_config;

typedef struct bsg_buffers {
  /* ---- aircraft state, fp64 [E*N] (bs.traf.* arrays) ---------------------------- */
  double *lat, *lon, *alt, *hdg, *tas, *cas, *vs, *ax;
  double *ap_trk, *selspd, *selalt, *selvs;   /* autopilot targets */
  int32_t *nav;                               /* bit0 swlnav, bits 8..15 active waypoint */
  double *gs, *trk;          /* ground speed / track (bs.traf.gs, .trk); required only while
                                a wind field is set (bsg_set_wind) -- without wind gs = tas
                                and trk = hdg, and these may be NULL */
  double *memo_cache;        /* optional [2*E*N + 4*E] scratch owned by the caller, initialised to
                                NaN: cross-step memo of the pure per-aircraft speed-schedule
                                functions (exact: the entries' keys are the aircraft's stored
                                selspd/selalt/tas/alt bits; the [E][4] tail is the ownship's
                                atmosphere keyed by altitude, see bsg_kernels.hip).  Re-fill it
                                with NaN after writing any aircraft-state buffer directly;
                                NULL disables it */
  /* ---- per-env state [E] ----------------------------------------------------------- */
  int32_t *step_count;       /* TimeLimit elapsed steps */
  int32_t *flags;            /* BSG_FLAG_* (zero-initialised by the caller) */
  uint32_t *episode;         /* episode counter (Philox counter word) */
  int32_t *wpt_reach;        /* merge_env.py:97; PlanWaypoint: bit k = waypoint k reached */
  int32_t *faf_reached;      /* merge_env.py:92 (info faf_reach) */
  int32_t *total_intrusions; /* info */
  double *total_reward;      /* info */
  double *drift_sum;         /* info average_drift numerator (count = step_count) */
  double *target_alt;        /* vertical/descent target altitude (m) */
  double *final_altitude;    /* vertical/descent info */
  double *env_wpt_lat;       /* HorizontalCR per-env waypoint (horizontal_cr_env.py:135-148) */
  double *env_wpt_lon;
  double *env_geom;          /* [E, bsg_geom_width] StaticObstacle obstacles + waypoint,
                                SectorCR sector polygon + aircraft count + waypoint,
                                PlanWaypoint 5 waypoint lat then 5 lon */
  double *env_aux;           /* [E, 4] StaticObstacle: waypoint distance (km) and drift (deg)
                                of the last observation, drift samples, crashed flag */
  /* ---- outputs --------------------------------------------------------------------- */
  float *obs;                /* [E, obs_dim] sorted-key flatten (gymnasium spaces.Dict order) */
  float *final_obs;          /* [E, obs_dim] terminal obs (SAME_STEP only; else may be NULL) */
  float *reward;             /* [E] */
  uint8_t *terminated;       /* [E] */
  uint8_t *truncated;        /* [E] */
  int32_t *topk;             /* [E, K] aircraft index of the K nearest intruders (Merge) */
  uint64_t *intr_mask;       /* [E] bit i: ownship-aircraft i intrusion this step */
  uint64_t *conf_mask;       /* [E, N] StateBased swconfl, bit j of row i (compute_cd) */
  uint64_t *los_mask;        /* [E, N] StateBased swlos, bit j of row i (compute_cd) */
  float *tcpamax;            /* [E, N] StateBased tcpamax (compute_cd) */
  float *min_sep;            /* [E] min StateBased dist (m) over the pairs inside the CD
                                horizon RPZ + 300 s * vrel; +inf if no pair is inside it,
                                so well-separated envs read +inf (compute_cd) */
  double *ep_info;           /* [E, 4] written when an episode ends: total_reward,
                                total_intrusions, faf_reach | final_altitude,
                                average_drift (Merge) -- the info dict at done
                                (merge_env.py:238-244, vertical_cr_env.py:203-211) */
  float *learner;            /* optional [E, obs_dim + 3]: obs, reward, terminated,
                                truncated as fp32 -- the per-step learner hand-off row that
                                the multi-GPU path all-gathers over RCCL (NULL = off) */
} bsg_buffers;

/* Wind field (bluesky_gym/wrappers/wind.py:8-24 -> bs.traf.wind.addpointvne): P points with
 * wind components constant in altitude (num_levels = 1) or sampled on the fixed altitude
 * axis (num_levels = BSG_WIND_NALT, level l at l*100 ft).  Interpolation: inverse distance
 * squared over the points (one point and one level: constant everywhere), linear between
 * altitude levels (docs/BLUESKY_SUBSET_SPEC.md §A.7).  All pointers are device pointers
 * owned by the caller; vnorth/veast are [num_levels][P] (m/s). */
typedef struct bsg_wind {
  int32_t num_points;        /* P >= 1; 0 turns the wind off */
  int32_t num_levels;        /* 1 or BSG_WIND_NALT */
  int32_t augment_obs;       /* 1: obs rows carry wind_u, wind_v (wind.py:18-24, 56-66) at
                                their sorted-key position; obs_dim grows by 2 */
  int32_t reserved;
  const double *lat, *lon;   /* [P] deg */
  const double *vnorth, *veast;
} bsg_wind;

typedef struct bsg_ctx bsg_ctx;

/* ABI version of the loaded library. */
int32_t bsg_abi_version(void);

/* Thread-local message of the last failing call ("" if none). */
const char* bsg_last_error(void);

/* Flat observation length for an env kind (sum of the Box sizes of the reference
 * observation_space: merge_env.py:59-74 -> 5+7K; vertical_cr_env.py:67-83 -> 4+7(N-1);
 * descent_env.py:53-60 -> 4; horizontal_cr_env.py:49-60 -> 3+5(N-1);
 * static_obstacle_env.py:61-71 -> 3+4*10; sector_cr_env.py:53-66 -> 3+7K;
 * plan_waypoint_env.py:50-56 -> 4*5). Negative on
 * invalid input.  A wind field with augment_obs adds 2 (bsg_ctx_obs_dim). */
int32_t bsg_obs_dim(int32_t env_kind, int32_t num_ac, int32_t num_ac_state);

/* Action width (merge_env.py:76, static_obstacle_env.py:73, sector_cr_env.py:68 -> 2;
 * vertical_cr_env.py:85 / descent_env.py:62 / horizontal_cr_env.py:62 /
 * plan_waypoint_env.py:59 -> 1). */
int32_t bsg_action_dim(int32_t env_kind);

/* Doubles per env of host-supplied spawn parameters for bsg_reset / bsg_step:
 *   Merge    [2N]      : (bearing deg, distance km) for aircraft 0..N-1, the
 *                        random.uniform draws of merge_env.py:115-116,150-151
 *   Vertical [2+4(N-1)]: alt_init, target_alt, then (dpsi, cpa, tlosh, dH) per intruder,
 *                        the np.random draws of vertical_cr_env.py:188-195,267-268
 *   Descent  [2]       : alt_init, target_alt (descent_env.py:170-171)
 *   Horizontal [3(N-1)+1]: (dpsi, cpa, tlosh) per intruder, then the waypoint distance
 *                        (km), the np.random draws of horizontal_cr_env.py:130-132,140
 *   StaticObstacle [202]: per obstacle (distance km, bearing deg, area NM^2, vertices,
 *                        16 uniform circle draws), then waypoint (distance km, bearing deg)
 *                        (static_obstacle_env.py:148-226)
 *   SectorCR [68+3N]   : aircraft count, vertices, 32 vertex lat, 32 vertex lon, ownship
 *                        waypoint lat/lon, then (lat, lon, hdg) per aircraft
 *                        (sector_cr_env.py:84-208)
 *   PlanWaypoint [10]  : 5 waypoint distances (km) then 5 bearings (deg) from the ownship,
 *                        the np.random draws of plan_waypoint_env.py:205-206 */
int32_t bsg_spawn_width(int32_t env_kind, int32_t num_ac);

/* Doubles per env of bsg_buffers.env_geom (0 for kinds without per-env geometry):
 * StaticObstacle 2 + 10*(6 + 2*16); SectorCR 4 + 2*32; PlanWaypoint 2*5. */
int32_t bsg_geom_width(int32_t env_kind, int32_t num_ac);

/* Replaces: gym.make(id) -> Env.__init__ (merge_env.py:54-101): validates the config
 * and binds a device.  No device memory is allocated. */
int32_t bsg_create(const bsg_config* cfg, bsg_ctx** out);
int32_t bsg_destroy(bsg_ctx* ctx);

/* Attach the caller-owned device buffers (non-owning). */
int32_t bsg_bind(bsg_ctx* ctx, const bsg_buffers* bufs);

/* Re-point only the optional learner-row buffer ([E, obs_dim + 3] fp32, NULL = none) of a
 * bound ctx, from the next launch on: the multi-GPU path double-buffers the rows it
 * all-gathers (bluesky_gym/parallel.py) and swaps them every step without re-binding.
 * Replaces nothing in the reference (its learner hand-off is SubprocVecEnv's pipe,
 * stable_baselines3 common/vec_env/subproc_vec_env.py). */
int32_t bsg_set_learner(bsg_ctx* ctx, float* learner_rows);

/* Lookahead (MergeEnv-v0 and VerticalCREnv-v0; NEXT_STEP or no autoreset; inactive while a
 * wind field is set).  Merge's intruders fly their LNAV route, Vertical's their creconfs
 * straight line, independently of the ownship and the action (merge_env.py:155-157,
 * vertical_cr_env.py:183-200; RESO OFF), so with a caller-owned scratch of
 * bsg_lookahead_bytes() bytes bound, every launch also propagates the intruders one RL
 * step ahead in extra workgroups, and the next step consumes that state instead of
 * integrating the intruders on its critical path (Merge, small batches: the scratch also
 * holds a cache of each env's next-episode creation positions, drawn ahead by idle waves).
 * Results are bit-identical to the inline path.  bsg_lookahead_bytes returns 0 when the
 * ctx cannot use it;
 * bsg_set_lookahead(ctx, NULL, 0) turns it off.  Binding, a wind change or calling
 * bsg_set_lookahead again restarts it from the state buffers (call it again after
 * writing aircraft state directly, as for memo_cache).  Replaces nothing in the reference
 * (a scheduling device: merge_env.py:136-137 / vertical_cr_env.py:287-289 run the substeps of
 * all aircraft). */
int64_t bsg_lookahead_bytes(const bsg_ctx* ctx);
int32_t bsg_set_lookahead(bsg_ctx* ctx, void* scratch, int64_t bytes);

/* Trajectory store (MergeEnv-v0 with the lookahead bound, NEXT_STEP autoreset, a TimeLimit of
 * 1..63 steps; device spawns).  A Merge intruder's whole episode depends only on (seed, env,
 * Philox episode counter) -- it spawns at merge_env.py:148-158 and flies LNAV with RESO OFF --
 * so the library flies future episodes ahead, every post-step state of every step and the
 * intruder pairs' conflict rows, on a stream of its own at the least priority (a few steps of
 * each episode per producer launch, one launch after the other), and the step
 * launch's lookahead copies the next step's entry instead of propagating ten substeps on its
 * critical path.  Same function of the same inputs: every output is bit-identical to the
 * inline path.  A reset with device spawns flies the new episodes on the caller's stream; a
 * launch with host spawn rows, a re-bind or a re-armed lookahead retires the stored episodes.
 * The caller owns the scratch (bsg_trajectory_bytes; 0 = unsupported configuration) and
 * keeps it until bsg_set_trajectory(ctx, NULL, 0, 0) or bsg_destroy, which wait for the
 * producer.  flags: BSG_TRAJ_SYNC (tests) runs the producers on the caller's stream. */
#define BSG_TRAJ_SYNC 1
int64_t bsg_trajectory_bytes(const bsg_ctx* ctx);
int32_t bsg_set_trajectory(bsg_ctx* ctx, void* scratch, int64_t bytes, int32_t flags);
/* out[0] store bound, out[1] producer launches issued, out[2] producer launches enqueued and not seen complete,
 * out[3] generation */
int32_t bsg_trajectory_info(const bsg_ctx* ctx, int64_t* out);

/* Replaces: Env.reset() (merge_env.py:103-130 + _gen_aircraft :148-158;
 * vertical_cr_env.py:258-281 + _generate_conflicts :183-200; descent_env.py:162-182).
 * env_mask: device u8 [E] (NULL = all envs).  spawn: device f64 [E, spawn_width]
 * (NULL = Philox draw keyed by (seed, env, episode)).  Writes obs. */
int32_t bsg_reset(bsg_ctx* ctx, const uint8_t* env_mask, const double* spawn, void* stream);

/* Replaces: Env.step(action) + TimeLimit (merge_env.py:132-146; vertical_cr_env.py:283-305;
 * descent_env.py:184-206).  actions: device f64 [E, action_dim].  spawn: optional
 * device f64 [E, spawn_width] used by autoresets in this step (NULL = Philox). */
int32_t bsg_step(bsg_ctx* ctx, const double* actions, const double* spawn, void* stream);

/* Replaces: WindFieldWrapper(env, lat, lon, vnorth, veast, alt, augment_obs)
 * (wind.py:8-24, addpointvne at :28): sets (or, with NULL / num_points 0, clears) the wind
 * field applied to every env of the batch from the next launch on.  Unbinds the ctx:
 * call bsg_bind again (gs/trk become required; obs rows may widen). */
int32_t bsg_set_wind(bsg_ctx* ctx, const bsg_wind* wind);

/* The env module's constants (MergeEnv-v0: merge_env.py:13-46), so that a caller that patches
 * them (the drop-in bluesky_gym.envs.merge_env reads its module globals at construction)
 * changes the device env as it would the reference: values[BSG_MERGE_NPARAMS] in the order
 * below (the reference's units: degrees, m/s, NM, km as merge_env.py compares them).  Each
 * defaults to the reference's value at bsg_create.  AC_SPD is bsg_config.kind_option.
 * Merge only; call before the first bsg_reset / bsg_step of the ctx (BSG_E_STATE after). */
enum { BSG_MP_D_HEADING = 0,          /* merge_env.py:27: +-deg of the HDG action and of the
                                          spawn bearings (:115, :150) */
       BSG_MP_D_SPEED,                /* :28: m/s of the SPD action */
       BSG_MP_INTRUSION_DISTANCE,     /* :19: NM, _check_intrusion */
       BSG_MP_DISTANCE_MARGIN,        /* :13: _check_waypoint (compared with the NM distance) */
       BSG_MP_REACH_REWARD,           /* :14 */
       BSG_MP_DRIFT_PENALTY,          /* :16 */
       BSG_MP_INTRUSION_PENALTY,      /* :17 */
       BSG_MP_SPAWN_DISTANCE_MIN,     /* :21-22: the ownship's spawn distance to the FAF */
       BSG_MP_SPAWN_DISTANCE_MAX,
       BSG_MP_INTRUDER_DISTANCE_MIN,  /* :24-25: the intruders' */
       BSG_MP_INTRUDER_DISTANCE_MAX,
       BSG_MERGE_NPARAMS };
int32_t bsg_set_params(bsg_ctx* ctx, const double* values, int32_t count);

/* Observation row length of this ctx (bsg_obs_dim + 2 with an augmenting wind field). */
int32_t bsg_ctx_obs_dim(const bsg_ctx* ctx);

/* Kernel-time instrumentation: record a HIP event pair on the launch stream around every
 * `enable`-th step/reset launch (1 = every launch, k = launches 0, k, 2k, ... after the
 * call; 0 = off).  An event pair adds ~8 us of stream serialisation to the launch it
 * brackets, so throughput runs sample (bench.py: every 10th).  bsg_step_timing returns
 * the summed elapsed ms and the number of timed launches since its last call
 * (synchronises on those events). */
int32_t bsg_set_timing(bsg_ctx* ctx, int32_t enable);
int32_t bsg_step_timing(bsg_ctx* ctx, double* total_ms, int32_t* launches);

/* Diagnostics: per-wave phase stamps (8 x u64 per workgroup: realtime start/end at 100 MHz,
 * shader-clock stamps after each phase, hardware XCC/CU ids) into a caller-owned device
 * buffer of grid_size*8 u64.  Only a library built with -DBSG_STAMPS=1 (make stamps)
 * writes them; otherwise returns BSG_E_UNSUPPORTED.  Never used on the measured path. */
int32_t bsg_set_stamps(bsg_ctx* ctx, void* device_buf);

/* Device policy: the weights of an SB3 SAC actor (MultiInputPolicy, net_arch [256, 256]:
 * latent_pi.0, latent_pi.2, mu, log_std; nn.Linear layout [out, in], fp32, device memory;
 * w1 16-byte aligned).  The caller owns them; a learner may update them in place. */
typedef struct bsg_sac_actor {
  int32_t obs_dim;           /* 1..256 */
  int32_t act_dim;           /* 1..4 */
  int32_t hidden;            /* must be 256 */
  int32_t reserved;
  const float *w0, *b0;      /* [hidden, obs_dim], [hidden] */
  const float *w1, *b1;      /* [hidden, hidden], [hidden] */
  const float *w_mu, *b_mu;  /* [act_dim, hidden], [act_dim] */
  const float *w_ls, *b_ls;  /* [act_dim, hidden], [act_dim] */
} bsg_sac_actor;

/* Replaces: model.predict(obs, deterministic=True) (reference main.py:54,
 * scripts/multi_processing_example.py:70) and the per-step action sampling of SB3 SAC's
 * collect_rollouts (Actor.action_log_prob, stable_baselines3 2.x sac/policies.py; the
 * library is not vendored in the reference) for a whole batch, as one kernel:
 * a = tanh(mu + exp(clamp(log_std, -20, 2)) * eps) with eps: device fp32 [E, act_dim]
 * standard normals (NULL = deterministic, a = tanh(mu)).  obs: device fp32 rows of
 * `obs_stride` floats (the step kernel's obs, or learner rows).  actions: device f64
 * [E, act_dim] (what bsg_step reads).  log_prob: optional device fp32 [E] (SB3's
 * log_prob with the tanh correction).  Asynchronous on `stream`; capturable in a graph. */
int32_t bsg_policy_sac(const bsg_sac_actor* actor, const float* obs, int32_t num_envs,
                       int32_t obs_stride, const float* eps, double* actions, float* log_prob,
                       void* stream);

/* ---- the multi-GPU learner-row all-gather (RCCL over xGMI) -----------------------------
 * Replaces: the reference's vectorisation is SubprocVecEnv (scripts/multi_processing_example
 * .py:51-53), one env per process feeding one learner; here every rank's shard of envs
 * hands its learner rows [n_local, obs+3] fp32 (bsg_set_learner) to every rank by one
 * all-gather per RL step.  RCCL is resolved at run time (the process's
 * librccl.so.1 -- torch's -- else ROCm's).  The gather runs on a comm-owned stream of the
 * greatest priority after the caller's work (overlapping the caller's next kernels);
 * completion is tracked per slot (a ring of BSG_COMM_SLOTS row buffers) through fence
 * events recorded every BSG_COMM_SLOTS/2 gathers, and bsg_comm_wait makes a stream wait for
 * a slot's last gather -- the consumer of the gathered rows, or the step that next
 * overwrites that slot's rows (a no-op when that stream already waited for a fence covering
 * it).  All calls asynchronous; errors in bsg_comm_last_error().
 * Environment: BSG_COMM_GRAPHS=1 (the gather as a replayed HIP graph), BSG_COMM_PROFILE=1
 * (host time per part, printed at destroy). */
#define BSG_COMM_ID_BYTES 128
#define BSG_COMM_SLOTS 16
typedef struct bsg_comm bsg_comm;
const char* bsg_comm_last_error(void);
/* rank 0 draws the id (ncclGetUniqueId) and broadcasts it to the other ranks */
int32_t bsg_comm_unique_id(uint8_t* id /* [BSG_COMM_ID_BYTES] */);
int32_t bsg_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device,
                        bsg_comm** out);
int32_t bsg_comm_destroy(bsg_comm* comm);
/* recv[nranks * count] <- every rank's send[count] (rank-major), on the comm's stream after
 * everything `stream` has enqueued so far; slot in [0, BSG_COMM_SLOTS) */
int32_t bsg_comm_all_gather(bsg_comm* comm, const float* send, float* recv, int64_t count,
                            int32_t slot, void* stream);
int32_t bsg_comm_wait(bsg_comm* comm, int32_t slot, void* stream);
/* What the communicator is: RCCL's own view of it (ncclCommCount / ncclCommUserRank -- a
 * multi-GPU run records them, so that a node run shows RCCL saw every rank) and the comm's
 * counters (gathers issued; with BSG_COMM_GRAPHS=1 the graph cache's hits and captures). */
typedef struct bsg_comm_info {
  int32_t nranks;        /* ncclCommCount */
  int32_t rank;          /* ncclCommUserRank */
  int32_t device;        /* the HIP device the comm was created on */
  int32_t use_graphs;
  int64_t gathers;       /* bsg_comm_all_gather calls (bsg_step_gather included) */
  int64_t graph_hits;    /* gathers replayed from the graph cache */
  int64_t graph_captures;/* gathers captured into a new graph */
  int64_t reduces;       /* bsg_comm_all_reduce calls */
} bsg_comm_info;
int32_t bsg_comm_get_info(const bsg_comm* comm, bsg_comm_info* out);
/* The data-parallel learner's gradient reduction (C5, BASELINE configs[4]: "DescentEnv-v0 +
 * SB3 SAC learner, 4096 envs on 8 GPUs"; the reference trains one SB3 SAC in one process,
 * scripts/descent_env_sac.py:25-34, so this is the N-rank form of its gradient step):
 * buf[count] fp32 <- the sum (op BSG_REDUCE_SUM) or mean (BSG_REDUCE_AVG) over the ranks of
 * every rank's buf, in place, as ncclAllReduce on `stream` itself (ordered after what
 * `stream` enqueued and before what it enqueues next), so a learner update that calls it
 * stays one stream -- and capturable into a HIP graph. */
#define BSG_REDUCE_SUM 0
#define BSG_REDUCE_AVG 1
int32_t bsg_comm_all_reduce(bsg_comm* comm, float* buf, int64_t count, int32_t op, void* stream);
/* One RL step of a shard and the gather of its learner rows in one call (the host side of
 * a C4 step: ~one launch instead of a wait, a pointer swap, a launch and a gather):
 * bsg_comm_wait(slot) [the gather that last read rows[slot]], learner rows <- rows,
 * bsg_step, bsg_comm_all_gather(rows -> gathered, num_envs * (obs_dim + 3), slot). */
int32_t bsg_step_gather(bsg_ctx* ctx, bsg_comm* comm, const double* actions, const double* spawn,
                        float* rows, float* gathered, int32_t slot, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BSG_H_ */
