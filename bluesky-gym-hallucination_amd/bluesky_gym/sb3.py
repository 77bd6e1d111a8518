"""Stable-Baselines3 VecEnv adapter (the consumer of the reference's only vectorisation,
scripts/multi_processing_example.py:51-53 -- SubprocVecEnv).

``SB3VecEnv`` keeps SB3's contract: immediate (SAME_STEP) autoreset, the terminal
observation in ``infos[i]["terminal_observation"]``, ``infos[i]["TimeLimit.truncated"]``,
and every env's info dict carries the reference's info keys (merge_env.py:238-244), which
the reference's CSVLoggerCallback (bluesky_gym/utils/logger.py:15-34) reads from
``infos[0]``.  SB3 is not required to import this module; when it is installed the
class subclasses ``stable_baselines3.common.vec_env.VecEnv``.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native as nat
from .vector import (BlueSkyVectorEnv, DescentVectorEnv, HorizontalCRVectorEnv, MergeVectorEnv,
                     PlanWaypointVectorEnv, SectorCRVectorEnv, StaticObstacleVectorEnv,
                     VerticalCRVectorEnv)

try:  # pragma: no cover
    from stable_baselines3.common.vec_env import VecEnv as _SB3Base
except ImportError:
    _SB3Base = object

VECTOR_ENVS = {"MergeEnv-v0": MergeVectorEnv, "VerticalCREnv-v0": VerticalCRVectorEnv,
               "DescentEnv-v0": DescentVectorEnv, "HorizontalCREnv-v0": HorizontalCRVectorEnv,
               "StaticObstacleEnv-v0": StaticObstacleVectorEnv,
               "SectorCREnv-v0": SectorCRVectorEnv, "PlanWaypointEnv-v0": PlanWaypointVectorEnv}


def episode_infos(venv: BlueSkyVectorEnv, dones, term, trunc):
    """Per-env info dicts after a SAME_STEP launch: the running info of every env, and for
    an env that finished (and was already respawned) its finished episode's info from
    ep_info (merge_env.py:238-244; vertical_cr_env.py:203-211; descent_env.py:119-126)."""
    b = venv.batch
    kind = venv.kind_cfg.kind
    cur = venv._infos(done=None)
    cur.pop("conflicts", None)
    keys = list(cur)
    ep = b.ep_info.cpu().numpy() if dones.any() else None
    infos = []
    for i in range(venv.num_envs):
        d = {k: cur[k][i].item() for k in keys}
        if dones[i]:
            d["total_reward"] = float(ep[i, 0])
            if kind == nat.ENV_MERGE:
                d["total_intrusions"] = int(ep[i, 1])
                d["faf_reach"] = int(ep[i, 2])
                d["average_drift"] = float(ep[i, 3])
            elif kind == nat.ENV_VERTICAL_CR:
                d["total_intrusions"] = int(ep[i, 1])
                d["final_altitude"] = float(ep[i, 2])
            elif kind in (nat.ENV_HORIZONTAL_CR, nat.ENV_SECTOR_CR):
                d["total_intrusions"] = int(ep[i, 1])
                d["average_drift"] = float(ep[i, 2])
            elif kind == nat.ENV_STATIC_OBSTACLE:
                d["waypoint_reached"] = int(ep[i, 1])
                d["crashed"] = int(ep[i, 2])
                d["average_drift"] = float(ep[i, 3])
            elif kind == nat.ENV_PLAN_WAYPOINT:
                d["waypoints_completed"] = int(ep[i, 2])
            else:
                d["final_altitude"] = float(ep[i, 2])
            d["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
        infos.append(d)
    return infos


class SB3VecEnv(_SB3Base):
    def __init__(self, env_id: str, num_envs: int, *, seed=0, device=None, **env_kwargs):
        self.venv: BlueSkyVectorEnv = VECTOR_ENVS[env_id](
            num_envs=num_envs, seed=seed, device=device, autoreset=nat.AUTORESET_SAME_STEP,
            **env_kwargs)
        self.num_envs = num_envs
        self.observation_space = self.venv.single_observation_space
        self.action_space = self.venv.single_action_space
        self.render_mode = None
        self._actions = None

    # ------------------------------------------------------------------ SB3 API
    def reset(self):
        obs, _ = self.venv.reset()
        return obs

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        a = self._actions
        a = a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a, np.float64))
        b = self.venv.batch
        obs_t, rew_t, term_t, trunc_t = self.venv.step_tensors(a)
        term = term_t.cpu().numpy().astype(bool)
        trunc = trunc_t.cpu().numpy().astype(bool)
        dones = term | trunc
        obs = self.venv.layout.split(obs_t.cpu().numpy())
        infos = self._infos(dones, term, trunc)
        if dones.any():
            fin = self.venv.layout.split(b.final_obs.cpu().numpy())
            for i in np.nonzero(dones)[0]:
                infos[i]["terminal_observation"] = {k: v[i] for k, v in fin.items()}
        return obs, rew_t.cpu().numpy().astype(np.float32), dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _infos(self, dones, term, trunc):
        return episode_infos(self.venv, dones, term, trunc)

    def close(self):
        self.venv.close()

    def seed(self, seed=None):
        return [None] * self.num_envs

    def get_attr(self, attr_name, indices=None):
        n = len(self._idx(indices))
        return [getattr(self.venv, attr_name, None)] * n

    def set_attr(self, attr_name, value, indices=None):
        setattr(self.venv, attr_name, value)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        raise NotImplementedError("per-env methods are not available on a device batch")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._idx(indices))

    def get_images(self):
        return [None] * self.num_envs

    def _idx(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices
