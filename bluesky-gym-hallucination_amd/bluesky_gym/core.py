"""DeviceBatch: E independent envs of one kind as device-resident SoA tensors, stepped by
libbsg.so.  PyTorch-ROCm provides device memory and the stream; all arithmetic runs in
the HIP kernels (csrc/bsg_kernels.hip).  There is no CPU fallback.
"""
from __future__ import annotations

import os

import ctypes as C

import torch

from . import _native as nat
from .config import EnvKindConfig

# torch's raw current-stream getter (an int handle; the public torch.cuda.current_stream()
# builds a Stream object per call); absent in some builds -> the public API
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)

F64_STATE = ("lat", "lon", "alt", "hdg", "tas", "cas", "vs", "ax",
             "ap_trk", "selspd", "selalt", "selvs")
I32_ENV = ("step_count", "flags", "wpt_reach", "faf_reached", "total_intrusions")
F64_ENV = ("total_reward", "drift_sum", "target_alt", "final_altitude")


class DeviceBatch:
    # auto lookahead up to this many envs per GPU: below it the launch leaves SIMDs idle
    # and the intruders' substeps are the critical path (C4 shards); DESIGN.md §3
    LOOKAHEAD_MAX_ENVS = 2048
    # auto trajectory store (MergeEnv) up to this many envs per GPU: its producer waves share
    # the SIMDs the step launch leaves idle (C4's 8- and 4-GPU shards); DESIGN.md §6
    TRAJECTORY_MAX_ENVS = 1024

    def __init__(self, cfg: EnvKindConfig, num_envs: int, *, autoreset=nat.AUTORESET_NEXT_STEP,
                 compute_cd=True, seed=0, device=None, learner=False, env_offset=0,
                 memo_cache=True, lookahead=None, trajectory=None):
        """lookahead: propagate the intruders (Merge, Vertical) one RL step ahead in extra workgroups
        (bsg_set_lookahead; bit-identical results).  None = on where the library supports
        it and the batch is small enough to leave SIMDs idle (LOOKAHEAD_MAX_ENVS); True /
        False force it."""
        if not torch.cuda.is_available():
            raise nat.BsgError("bluesky_gym needs a HIP device (MI355X); none is visible")
        self.lib = nat.load_library()
        self.cfg = cfg
        self.E = int(num_envs)
        self.N = cfg.num_ac
        self.K = cfg.num_ac_state
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index or 0)
        self._dev_index = self.device.index
        self.autoreset = autoreset
        self.want_learner = bool(learner)
        self.want_memo = bool(memo_cache)
        self.compute_cd = bool(compute_cd) and cfg.num_ac > 1   # single-aircraft kinds: no CD
        self.obs_dim = self.lib.bsg_obs_dim(cfg.kind, cfg.num_ac, cfg.num_ac_state)
        if self.obs_dim < 0:
            raise nat.BsgError(f"invalid env config {cfg}")
        self.act_dim = self.lib.bsg_action_dim(cfg.kind)
        self.spawn_width = self.lib.bsg_spawn_width(cfg.kind, cfg.num_ac)
        self.env_offset = int(env_offset)
        self.seed = int(seed)
        self.wind = None
        self.wind_augment = False
        ccfg = cfg.to_c(self.E, autoreset, self.compute_cd, seed, self.device.index, env_offset)
        ctx = C.c_void_p()
        nat.check(self.lib.bsg_create(C.byref(ccfg), C.byref(ctx)), "bsg_create")
        self._ctx = ctx
        if getattr(cfg, "params", ()):
            pv = (C.c_double * len(cfg.params))(*cfg.params)
            nat.check(self.lib.bsg_set_params(ctx, pv, len(cfg.params)), "bsg_set_params")
        self._alloc()
        self._bind()
        self.lookahead = False
        self._la_buf = None
        nbytes = int(self.lib.bsg_lookahead_bytes(self._ctx))
        want = (lookahead if lookahead is not None
                else self.E <= self.LOOKAHEAD_MAX_ENVS)
        if want and nbytes > 0:
            self._la_buf = torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=self.device)
            nat.check(self.lib.bsg_set_lookahead(self._ctx, C.c_void_p(self._la_buf.data_ptr()),
                                                 nbytes), "bsg_set_lookahead")
            self.lookahead = True
        elif lookahead:
            raise nat.BsgError("lookahead: MergeEnv / VerticalCREnv with NEXT_STEP (or no) "
                               "autoreset only")
        # trajectory store (bsg_set_trajectory): MergeEnv's future episodes flown ahead on a
        # low-priority stream, copied by the lookahead (bit-identical).  Opt-in: True / "sync"
        # (the producers on the launch stream, tests); None = BSG_TRAJECTORY=1 turns it on for
        # the lookahead's Merge batches up to TRAJECTORY_MAX_ENVS.  Off by default: its
        # concurrent producers slow the step launches they share SIMDs with by more than the
        # copies save in steady state (profiles/r06/trajectory/)
        self.trajectory = False
        self._tj_buf = None
        tbytes = int(self.lib.bsg_trajectory_bytes(self._ctx)) if self.lookahead else 0
        want_tj = (trajectory if trajectory is not None
                   else self.E <= self.TRAJECTORY_MAX_ENVS and os.environ.get("BSG_TRAJECTORY", "0") == "1")
        if want_tj and tbytes > 0:
            self._tj_buf = torch.empty((tbytes + 7) // 8, dtype=torch.float64, device=self.device)
            flags = nat.TRAJ_SYNC if trajectory == "sync" else 0
            nat.check(self.lib.bsg_set_trajectory(self._ctx, C.c_void_p(self._tj_buf.data_ptr()),
                                                  tbytes, flags), "bsg_set_trajectory")
            self.trajectory = True
        elif trajectory:
            raise nat.BsgError("trajectory: MergeEnv with the lookahead, NEXT_STEP autoreset and a "
                               "TimeLimit of 1..63 steps only")

    # ------------------------------------------------------------------ buffers
    def _alloc(self):
        d, E, N = self.device, self.E, self.N
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=d)
        self.state = {k: z((E, N), torch.float64) for k in F64_STATE}
        self.state["nav"] = z((E, N), torch.int32)
        # cross-step memo of the speed schedule (csrc: memo_load/memo_store); NaN = no entry
        # [2][E*N] per-aircraft entries, then [E][4] ownship atmosphere (csrc: memo_*, oat)
        self.memo_cache = torch.full((2 * E * N + 4 * E,), float("nan"), dtype=torch.float64, device=d) \
            if self.want_memo else None
        self.envs = {k: z((E,), torch.int32) for k in I32_ENV}
        self.envs["episode"] = z((E,), torch.int32)     # uint32 on the device side
        self.envs.update({k: z((E,), torch.float64) for k in F64_ENV})
        self.obs = z((E, self.obs_dim), torch.float32)
        self.final_obs = z((E, self.obs_dim), torch.float32) \
            if self.autoreset == nat.AUTORESET_SAME_STEP else None
        self.reward = z((E,), torch.float32)
        self.terminated = z((E,), torch.uint8)
        self.truncated = z((E,), torch.uint8)
        self.topk = z((E, max(self.K, 1)), torch.int32) if self.cfg.kind == nat.ENV_MERGE else None
        self.intr_mask = z((E,), torch.int64)
        self.ep_info = z((E, 4), torch.float64)
        if self.cfg.kind == nat.ENV_HORIZONTAL_CR:
            self.envs["env_wpt_lat"] = z((E,), torch.float64)
            self.envs["env_wpt_lon"] = z((E,), torch.float64)
        gw = self.lib.bsg_geom_width(self.cfg.kind, N)
        if gw > 0:
            self.envs["env_geom"] = z((E, gw), torch.float64)
        if self.cfg.kind == nat.ENV_STATIC_OBSTACLE:
            self.envs["env_aux"] = z((E, 4), torch.float64)
        # learner hand-off rows [obs, reward, terminated, truncated] (RCCL all-gather payload)
        self.learner = z((E, self.obs_dim + 3), torch.float32) if self.want_learner else None
        if self.compute_cd:
            self.conf_mask = z((E, N), torch.int64)
            self.los_mask = z((E, N), torch.int64)
            self.tcpamax = z((E, N), torch.float32)
            self.min_sep = z((E,), torch.float32)
        else:
            self.conf_mask = self.los_mask = self.tcpamax = self.min_sep = None

    def set_wind(self, table, augment_obs=False):
        """Apply a wind field (bluesky_gym.wind.WindTable, or None to clear) to every env
        from the next launch on (wrappers/wind.py).  augment_obs widens the obs rows by
        wind_u / wind_v; the obs buffers are reallocated then (call reset afterwards)."""
        d = self.device
        w = nat.BsgWind()
        if table is not None:
            self._wind_tabs = [torch.as_tensor(a, dtype=torch.float64).to(d).contiguous()
                               for a in (table.lat, table.lon, table.vnorth, table.veast)]
            w.num_points = table.num_points
            w.num_levels = table.num_levels
            w.augment_obs = int(bool(augment_obs))
            w.lat, w.lon, w.vnorth, w.veast = (C.cast(C.c_void_p(t.data_ptr()), nat._dp)
                                               for t in self._wind_tabs)
            if "gs" not in self.state:
                # without wind gs = tas and trk = hdg exactly (Traffic.update_groundspeed)
                self.state["gs"] = self.state["tas"].clone()
                self.state["trk"] = self.state["hdg"].clone()
        else:
            self._wind_tabs = None
        nat.check(self.lib.bsg_set_wind(self._ctx, C.byref(w)), "bsg_set_wind")
        od = self.lib.bsg_ctx_obs_dim(self._ctx)
        if od != self.obs_dim:
            self.obs_dim = od
            z = lambda shape: torch.zeros(shape, dtype=torch.float32, device=d)
            self.obs = z((self.E, od))
            if self.final_obs is not None:
                self.final_obs = z((self.E, od))
            if self.learner is not None:
                self.learner = z((self.E, od + 3))
        self.wind = table
        self.wind_augment = table is not None and bool(augment_obs)
        self._bind()

    def _bind(self):
        b = nat.BsgBuffers()
        src = dict(self.state)
        src.update(self.envs)
        src.update(memo_cache=self.memo_cache)
        src.update(obs=self.obs, final_obs=self.final_obs, reward=self.reward,
                   terminated=self.terminated, truncated=self.truncated, topk=self.topk,
                   intr_mask=self.intr_mask, conf_mask=self.conf_mask, los_mask=self.los_mask,
                   tcpamax=self.tcpamax, min_sep=self.min_sep, ep_info=self.ep_info,
                   learner=self.learner)
        for name, ptype in nat.BUFFER_FIELDS:
            t = src.get(name)
            setattr(b, name, C.cast(C.c_void_p(t.data_ptr()), ptype) if t is not None
                    else ptype())
        self._bufs = b
        nat.check(self.lib.bsg_bind(self._ctx, C.byref(b)), "bsg_bind")

    def invalidate_caches(self):
        """After writing self.state directly: the memo cache and the lookahead restart
        from the buffers (bsg.h: memo_cache, bsg_set_lookahead)."""
        if self.memo_cache is not None:
            self.memo_cache.fill_(float("nan"))
        if self._la_buf is not None:
            nat.check(self.lib.bsg_set_lookahead(self._ctx, C.c_void_p(self._la_buf.data_ptr()),
                                                 self._la_buf.numel() * 8), "bsg_set_lookahead")

    def set_learner(self, rows: torch.Tensor | None):
        """Point the kernel's learner-row output at `rows` ([E, obs_dim + 3] fp32 on this
        device, or None) without re-binding the other buffers (bsg_set_learner)."""
        if rows is not None:
            if (rows.dtype != torch.float32 or rows.device != self.device or not rows.is_contiguous()
                    or tuple(rows.shape) != (self.E, self.obs_dim + 3)):
                raise nat.BsgError(f"learner rows must be contiguous fp32 [{self.E}, {self.obs_dim + 3}] "
                                   f"on {self.device}")
        nat.check(self.lib.bsg_set_learner(self._ctx, C.c_void_p(rows.data_ptr()) if rows is not None
                                           else None), "bsg_set_learner")
        self.learner = rows

    def _stream(self):
        # the caller's current stream on this device (the raw handle getter skips building a
        # torch.cuda.Stream object: ~2.4 -> ~0.3 us of host time per launch)
        if _raw_stream is not None:
            return C.c_void_p(_raw_stream(self._dev_index))
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ API
    def reset(self, env_mask: torch.Tensor | None = None, spawn: torch.Tensor | None = None):
        """Env.reset for the envs in env_mask (u8/bool [E] on device; None = all).
        spawn: f64 [E, spawn_width] on device (parity mode) or None (device Philox)."""
        m = None
        if env_mask is not None:
            m = env_mask.to(device=self.device, dtype=torch.uint8).contiguous()
        sp = self._spawn_arg(spawn)
        nat.check(self.lib.bsg_reset(self._ctx, C.c_void_p(m.data_ptr()) if m is not None else None,
                                     C.c_void_p(sp.data_ptr()) if sp is not None else None,
                                     self._stream()), "bsg_reset")
        self._keep = (m, sp)
        return self.obs

    def step(self, actions: torch.Tensor, spawn: torch.Tensor | None = None):
        """One RL step of every env.  actions: [E, act_dim] (any float dtype/device; kept
        as f64 on device).  Returns (obs, reward, terminated, truncated) device views."""
        a = actions
        if a.dtype != torch.float64 or a.device != self.device or not a.is_contiguous():
            a = a.to(device=self.device, dtype=torch.float64).contiguous()
        if a.shape != (self.E, self.act_dim):
            a = a.reshape(self.E, self.act_dim)
        sp = self._spawn_arg(spawn)
        nat.check(self.lib.bsg_step(self._ctx, C.c_void_p(a.data_ptr()),
                                    C.c_void_p(sp.data_ptr()) if sp is not None else None,
                                    self._stream()), "bsg_step")
        self._keep = (a, sp)
        return self.obs, self.reward, self.terminated, self.truncated

    def _spawn_arg(self, spawn):
        if spawn is None:
            return None
        sp = spawn.to(device=self.device, dtype=torch.float64).contiguous()
        if sp.shape != (self.E, self.spawn_width):
            raise nat.BsgError(f"spawn must be [{self.E}, {self.spawn_width}], got {tuple(sp.shape)}")
        return sp

    def set_timing(self, every: int | bool):
        """HIP event pair around every `every`-th launch (True = 1 = every launch, 0 = off)."""
        nat.check(self.lib.bsg_set_timing(self._ctx, int(every)), "bsg_set_timing")

    def step_timing(self):
        """(total kernel ms, launches) since the last call (HIP events on the launch stream)."""
        ms = C.c_double()
        n = C.c_int32()
        nat.check(self.lib.bsg_step_timing(self._ctx, C.byref(ms), C.byref(n)), "bsg_step_timing")
        return ms.value, n.value

    def info(self):
        """Per-env running info (device tensors)."""
        return dict(total_reward=self.envs["total_reward"],
                    total_intrusions=self.envs["total_intrusions"],
                    faf_reach=self.envs["faf_reached"],
                    drift_sum=self.envs["drift_sum"], step_count=self.envs["step_count"],
                    final_altitude=self.envs["final_altitude"])

    def trajectory_info(self) -> dict:
        """bsg_trajectory_info and the lookahead's copies from the store per env (the store's
        diagnostic counters, tests/test_gpu_trajectory.py)."""
        out = (C.c_int64 * 4)()
        nat.check(self.lib.bsg_trajectory_info(self._ctx, out), "bsg_trajectory_info")
        copies = (self._tj_buf[:self.E].view(torch.int64).cpu() if self._tj_buf is not None
                  else torch.zeros(self.E, dtype=torch.int64))
        return {"bound": int(out[0]), "producer_launches": int(out[1]), "producer_outstanding": int(out[2]),
                "generation": int(out[3]), "copies": copies}

    def close(self):
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            self.lib.bsg_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
