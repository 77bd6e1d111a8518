"""Gymnasium VectorEnv front-ends of the device batch (the ``vector_entry_point`` of
MergeEnv-v0 / VerticalCREnv-v0 / DescentEnv-v0 / HorizontalCREnv-v0 / StaticObstacleEnv-v0 /
SectorCREnv-v0 / PlanWaypointEnv-v0, registered by ``register_envs``).

``gym.make_vec("MergeEnv-v0", num_envs=4096, vectorization_mode="vector_entry_point",
num_ac=32)`` returns a :class:`MergeVectorEnv` whose E envs live on one HIP device and
advance with one kernel launch per ``step``.

Autoreset follows Gymnasium >= 1.0's default NEXT_STEP mode: the step after a
terminated/truncated step resets that env (its action is ignored, reward 0).
Observations come back as the reference's Dict of float64 arrays, batched [E, k];
``step_tensors`` returns the device-resident fp32 views for zero-copy learners.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _gym, _native as nat, areas, config as cfgmod, spawn as spawnmod
from .core import DeviceBatch
from .obs_layout import ObsLayout

_INFO_KEYS = {
    nat.ENV_MERGE: ("total_reward", "faf_reach", "average_drift", "total_intrusions"),
    nat.ENV_VERTICAL_CR: ("total_reward", "total_intrusions", "final_altitude"),
    nat.ENV_DESCENT: ("total_reward", "final_altitude"),
    nat.ENV_HORIZONTAL_CR: ("total_reward", "total_intrusions", "average_drift"),
    nat.ENV_STATIC_OBSTACLE: ("total_reward", "waypoint_reached", "crashed", "average_drift"),
    nat.ENV_SECTOR_CR: ("total_reward", "total_intrusions", "average_drift"),
    nat.ENV_PLAN_WAYPOINT: ("total_reward", "waypoints_completed"),
}


class BlueSkyVectorEnv(_gym.VectorEnv):
    """E independent envs of one kind on one device."""

    metadata = {"autoreset_mode": "NextStep", "render_modes": []}

    def __init__(self, kind_cfg: cfgmod.EnvKindConfig, num_envs: int, *, device=None, seed=0,
                 compute_cd=True, spawn="device", autoreset=nat.AUTORESET_NEXT_STEP,
                 env_offset=0, learner=False):
        self.kind_cfg = kind_cfg
        self.num_envs = int(num_envs)
        self.device = device
        self.compute_cd = compute_cd
        self.spawn_mode = spawn
        self.autoreset = autoreset
        self.env_offset = env_offset
        self.learner = learner
        self.layout = ObsLayout(kind_cfg.kind, kind_cfg.num_ac, kind_cfg.num_ac_state)
        self.single_observation_space = self.layout.observation_space(_gym.spaces)
        act = 2 if kind_cfg.kind in (nat.ENV_MERGE, nat.ENV_STATIC_OBSTACLE, nat.ENV_SECTOR_CR) else 1
        self.single_action_space = _gym.spaces.Box(-1, 1, shape=(act,), dtype=np.float64)
        self.observation_space = _gym.spaces.Dict(
            {k: _gym.spaces.Box(-np.inf, np.inf, shape=(self.num_envs, n), dtype=np.float64)
             for k, n in self.layout.sizes.items()})
        self.action_space = _gym.spaces.Box(-1, 1, shape=(self.num_envs, act), dtype=np.float64)
        if spawn == "host" and autoreset == nat.AUTORESET_SAME_STEP:
            # SAME_STEP resets inside the step kernel, before the host knows which envs end;
            # host rows (reference-order RNG per env) can only be supplied for NEXT_STEP
            raise ValueError("spawn='host' needs NEXT_STEP autoreset (SAME_STEP respawns on the "
                             "device inside the step); use spawn='device' with SAME_STEP")
        self._seed = seed
        self._host_rngs = None
        self._wind = None
        self.batch = self._new_batch(seed)

    def set_wind(self, table, augment_obs=False):
        """Wind field for every env of the batch (bluesky_gym.wrappers.wind)."""
        k = self.kind_cfg
        self._wind = (table, augment_obs)
        self.batch.set_wind(table, augment_obs)
        self.layout = ObsLayout(k.kind, k.num_ac, k.num_ac_state, wind=self.batch.wind_augment)
        self.single_observation_space = self.layout.observation_space(_gym.spaces)
        self.observation_space = _gym.spaces.Dict(
            {key: _gym.spaces.Box(-np.inf, np.inf, shape=(self.num_envs, n), dtype=np.float64)
             for key, n in self.layout.sizes.items()})

    def _new_batch(self, seed):
        return DeviceBatch(self.kind_cfg, self.num_envs, autoreset=self.autoreset,
                           compute_cd=self.compute_cd, seed=seed, device=self.device,
                           learner=self.learner, env_offset=self.env_offset)

    # step_tensors() is the asynchronous device path: it only records the SectorCR overflow
    # flag on the device and reads it back every OVERFLOW_CHECK_EVERY calls (and in step()
    # / reset(), which copy to the host anyway), so it adds no per-step host sync.
    OVERFLOW_CHECK_EVERY = 64

    def _note_overflow(self):
        """Device-side: OR this launch's SectorCR spawn-overflow flags into a sticky
        per-env mask (no host sync)."""
        if self.kind_cfg.kind != nat.ENV_SECTOR_CR:
            return
        over = (self.batch.envs["flags"] & nat.FLAG_SPAWN_OVERFLOW) != 0
        prev = getattr(self, "_over", None)
        self._over = over if prev is None or prev.shape != over.shape else prev | over

    def _check_overflow(self, pending_only=False):
        """SectorCR: an episode that drew more aircraft than the capacity raises, as the
        host-spawn path does (bsg.h BSG_FLAG_SPAWN_OVERFLOW; sector_cr_env.py:95-100).
        pending_only: only what step_tensors() noted since the last check (reset / close:
        the flag of an overflow already raised persists in the env's flags)."""
        if self.kind_cfg.kind != nat.ENV_SECTOR_CR:
            return
        if not pending_only:
            self._note_overflow()
        over, self._over = getattr(self, "_over", None), None
        if over is not None and bool(over.any()):
            e = int(torch.nonzero(over)[0, 0])
            raise RuntimeError(f"SectorCR env {e}: the episode drew more aircraft than "
                               f"num_ac={self.kind_cfg.num_ac}; construct with a larger num_ac")

    # ---------------------------------------------------------------- spawns
    def _host_spawn(self, mask=None):
        """Per-env host RNG streams consuming draws like the reference (spawn='host')."""
        if self._host_rngs is None:
            ss = np.random.SeedSequence(self._seed)
            self._host_rngs = [np.random.RandomState(s.generate_state(1)[0])
                               for s in ss.spawn(self.num_envs)]
        k = self.kind_cfg
        rows = []
        for e in range(self.num_envs):
            if mask is not None and not mask[e]:
                rows.append(np.zeros(self.batch.spawn_width))
                continue
            rs = self._host_rngs[e]
            if k.kind == nat.ENV_MERGE:
                rows.append(spawnmod.merge_spawn(k.num_ac, rs))
            elif k.kind == nat.ENV_VERTICAL_CR:
                rows.append(spawnmod.vertical_spawn(k.num_ac - 1, rs))
            elif k.kind == nat.ENV_HORIZONTAL_CR:
                rows.append(spawnmod.horizontal_spawn(k.num_ac - 1, rs))
            elif k.kind == nat.ENV_STATIC_OBSTACLE:
                rows.append(areas.static_spawn(rs))
            elif k.kind == nat.ENV_SECTOR_CR:
                rows.append(areas.sector_spawn(k.num_ac, rs,
                                               "normal" if k.kind_option == 0 else "uniform"))
            elif k.kind == nat.ENV_PLAN_WAYPOINT:
                rows.append(spawnmod.plan_spawn(rs))
            else:
                rows.append(spawnmod.descent_spawn(rs))
        return torch.from_numpy(np.stack(rows))

    # ---------------------------------------------------------------- API
    def reset(self, *, seed=None, options=None):
        """Gymnasium reset.  reset(seed=s) always restarts from s -- fresh host RNG streams
        and episode counters (the Philox key) -- so two resets with the same seed give the
        same episodes; reset() without a seed continues the streams."""
        # an overflow flagged by step_tensors() calls since the last check raises here at the
        # latest (the rebuild below would drop the sticky mask)
        self._check_overflow(pending_only=True)
        if seed is not None:
            self._seed = seed
            self._host_rngs = None
            learner = self.batch.learner
            self.batch.close()
            self.batch = self._new_batch(seed)
            if self.learner and learner is not None:
                self.batch.set_learner(learner)
            if self._wind is not None:
                self.batch.set_wind(*self._wind)
        sp = self._host_spawn() if self.spawn_mode == "host" else None
        self.batch.reset(spawn=sp)
        self._check_overflow()
        return self.layout.split(self.batch.obs.cpu().numpy()), self._infos(done=None)

    def step_tensors(self, actions):
        """Device path: actions [E, A] (torch, any device) -> device views
        (obs fp32 [E, O], reward fp32 [E], terminated u8 [E], truncated u8 [E]).

        SectorCR capacity overflow (an episode drawing more than num_ac aircraft): this
        path adds no host sync, so the flag is read back only every OVERFLOW_CHECK_EVERY
        calls -- an overflowed episode can run up to that many steps with missing aircraft
        before the RuntimeError.  step(), reset() and close() check the sticky flag, so the
        error is never lost."""
        sp = None
        if self.spawn_mode == "host":
            pend = self.batch.envs["flags"].cpu().numpy() & 1
            sp = self._host_spawn(pend.astype(bool)) if pend.any() else None
        out = self.batch.step(actions, spawn=sp)
        self._since_check = getattr(self, "_since_check", 0) + 1
        if self._since_check >= self.OVERFLOW_CHECK_EVERY:
            self._since_check = 0
            self._check_overflow()
        else:
            self._note_overflow()
        return out

    def step(self, actions):
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions, np.float64))
        obs, rew, term, trunc = self.step_tensors(a)
        self._check_overflow()                   # the host copies below sync anyway
        term_np = term.cpu().numpy().astype(bool)
        trunc_np = trunc.cpu().numpy().astype(bool)
        return (self.layout.split(obs.cpu().numpy()), rew.cpu().numpy().astype(np.float64),
                term_np, trunc_np, self._infos(done=term_np | trunc_np))

    def _infos(self, done):
        """Gymnasium dict-of-arrays infos: the reference's per-env info dict
        (merge_env.py:238-244; vertical_cr_env.py:203-211; descent_env.py:119-126;
        horizontal_cr_env.py:215-223)."""
        b = self.batch
        tr = b.envs["total_reward"].cpu().numpy()
        out = {}
        kind = self.kind_cfg.kind
        if kind == nat.ENV_MERGE:
            cnt = b.envs["step_count"].cpu().numpy()
            with np.errstate(invalid="ignore", divide="ignore"):
                avg = b.envs["drift_sum"].cpu().numpy() / cnt
            out = {"total_reward": tr, "faf_reach": b.envs["faf_reached"].cpu().numpy(),
                   "average_drift": np.where(cnt > 0, avg, np.nan),
                   "total_intrusions": b.envs["total_intrusions"].cpu().numpy()}
        elif kind == nat.ENV_VERTICAL_CR:
            out = {"total_reward": tr, "total_intrusions": b.envs["total_intrusions"].cpu().numpy(),
                   "final_altitude": b.envs["final_altitude"].cpu().numpy()}
        elif kind == nat.ENV_STATIC_OBSTACLE:
            aux = b.envs["env_aux"].cpu().numpy()
            with np.errstate(invalid="ignore", divide="ignore"):
                avg = b.envs["drift_sum"].cpu().numpy() / aux[:, 2]
            out = {"total_reward": tr, "waypoint_reached": b.envs["wpt_reach"].cpu().numpy(),
                   "crashed": aux[:, 3].astype(np.int32),
                   "average_drift": np.where(aux[:, 2] > 0, avg, np.nan)}
        elif kind in (nat.ENV_HORIZONTAL_CR, nat.ENV_SECTOR_CR):
            cnt = b.envs["step_count"].cpu().numpy()
            with np.errstate(invalid="ignore", divide="ignore"):
                avg = b.envs["drift_sum"].cpu().numpy() / cnt
            out = {"total_reward": tr, "total_intrusions": b.envs["total_intrusions"].cpu().numpy(),
                   "average_drift": np.where(cnt > 0, avg, np.nan)}
        elif kind == nat.ENV_PLAN_WAYPOINT:
            wr = b.envs["wpt_reach"].cpu().numpy()
            done_cnt = sum((wr >> k) & 1 for k in range(5))
            out = {"total_reward": tr, "waypoints_completed": done_cnt.astype(np.int32)}
        else:
            out = {"total_reward": tr, "final_altitude": b.envs["final_altitude"].cpu().numpy()}
        if b.compute_cd:
            out["conflicts"] = (b.conf_mask.cpu().numpy() != 0).sum(axis=1)
        if done is not None:
            out["_final"] = done
        return out

    def close(self):
        try:
            if getattr(self.batch, "_ctx", None) is not None and self.batch._ctx.value:
                self._check_overflow(pending_only=True)
        finally:
            self.batch.close()


class MergeVectorEnv(BlueSkyVectorEnv):
    def __init__(self, num_envs=1, num_ac=20, num_ac_state=5, action_frequency=10, simdt=5.0,
                 max_episode_steps=50, **kw):
        super().__init__(cfgmod.merge_config(num_ac, num_ac_state, action_frequency, simdt,
                                             max_episode_steps or 0), num_envs, **kw)


class VerticalCRVectorEnv(BlueSkyVectorEnv):
    def __init__(self, num_envs=1, num_intruders=5, action_frequency=30, simdt=1.0,
                 max_episode_steps=300, num_ac=None, **kw):
        if num_ac is not None:
            num_intruders = num_ac - 1
        super().__init__(cfgmod.vertical_config(num_intruders, action_frequency, simdt,
                                                max_episode_steps or 0), num_envs, **kw)


class HorizontalCRVectorEnv(BlueSkyVectorEnv):
    def __init__(self, num_envs=1, num_intruders=5, action_frequency=10, simdt=5.0,
                 max_episode_steps=300, num_ac=None, **kw):
        if num_ac is not None:
            num_intruders = num_ac - 1
        super().__init__(cfgmod.horizontal_config(num_intruders, action_frequency, simdt,
                                                  max_episode_steps or 0), num_envs, **kw)


class StaticObstacleVectorEnv(BlueSkyVectorEnv):
    def __init__(self, num_envs=1, action_frequency=10, simdt=1.0, max_episode_steps=100, **kw):
        kw.pop("compute_cd", None)
        super().__init__(cfgmod.static_config(action_frequency, simdt, max_episode_steps or 0),
                         num_envs, compute_cd=False, **kw)


class SectorCRVectorEnv(BlueSkyVectorEnv):
    def __init__(self, num_envs=1, num_ac=32, action_frequency=5, simdt=1.0, max_episode_steps=200,
                 ac_density_mode="normal", **kw):
        super().__init__(cfgmod.sector_config(num_ac, action_frequency, simdt, max_episode_steps or 0,
                                              ac_density_mode), num_envs, **kw)


class DescentVectorEnv(BlueSkyVectorEnv):
    def __init__(self, num_envs=1, action_frequency=30, simdt=1.0, max_episode_steps=300, **kw):
        kw.pop("compute_cd", None)
        super().__init__(cfgmod.descent_config(action_frequency, simdt, max_episode_steps or 0),
                         num_envs, compute_cd=False, **kw)


class PlanWaypointVectorEnv(BlueSkyVectorEnv):
    """PlanWaypointEnv-v0 (plan_waypoint_env.py): five waypoints per episode around the
    ownship; like the reference, a reset after a truncation keeps the aircraft where it is
    (bsg.h BSG_FLAG_AC_PRESENT)."""

    def __init__(self, num_envs=1, action_frequency=10, simdt=1.0, max_episode_steps=300, **kw):
        kw.pop("compute_cd", None)
        super().__init__(cfgmod.plan_waypoint_config(action_frequency, simdt, max_episode_steps or 0),
                         num_envs, compute_cd=False, **kw)
