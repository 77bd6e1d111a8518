"""Single-env views (num_envs = 1) of the device batch with the reference's gym.Env
contract: ``reset(seed, options) -> (obs dict of float64 arrays, info)`` and
``step(action) -> (obs, reward: float, terminated: int 0/1, truncated: False, info)``.

Spawns consume Python ``random`` (Merge) / legacy ``np.random`` (Vertical, Descent)
exactly like the reference (merge_env.py:115-116,150-151; vertical_cr_env.py:188-195,
267-268; descent_env.py:170-171), so seeding those generators reproduces the
reference's episodes.  Rendering (pygame) is out of scope.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import _gym, _native as nat
from ..core import DeviceBatch
from ..obs_layout import ObsLayout


class SingleEnvBase(_gym.Env):
    metadata = {"render_modes": ["rgb_array", "human"], "render_fps": 120}

    def _init_batch(self, kind_cfg, render_mode, device, compute_cd):
        assert render_mode is None or render_mode in self.metadata["render_modes"]
        self.render_mode = render_mode
        self.kind_cfg = kind_cfg
        self.layout = ObsLayout(kind_cfg.kind, kind_cfg.num_ac, kind_cfg.num_ac_state)
        self.observation_space = self.layout.observation_space(_gym.spaces)
        self.batch = DeviceBatch(kind_cfg, 1, autoreset=nat.AUTORESET_NONE,
                                 compute_cd=compute_cd, device=device)
        self.action_space = _gym.spaces.Box(-1, 1, shape=(self.batch.act_dim,), dtype=np.float64)

    def set_wind(self, table, augment_obs=False):
        """Wind field for this env (bluesky_gym.wrappers.wind.WindFieldWrapper)."""
        k = self.kind_cfg
        self.batch.set_wind(table, augment_obs)
        self.layout = ObsLayout(k.kind, k.num_ac, k.num_ac_state, wind=self.batch.wind_augment)
        self.observation_space = self.layout.observation_space(_gym.spaces)

    def _spawn(self):
        raise NotImplementedError

    def _obs(self):
        return self.layout.split(self.batch.obs.cpu().numpy()[0])

    def reset(self, seed=None, options=None):
        super().reset(seed=seed)
        sp = torch.from_numpy(self._spawn()[None, :])
        self.batch.reset(spawn=sp)
        obs = self._obs()
        return obs, self._info()

    def step(self, action):
        a = torch.as_tensor(np.asarray(action, np.float64)).reshape(1, -1)
        self.batch.step(a)
        obs = self._obs()
        reward = float(self.batch.reward.cpu().numpy()[0])
        terminated = int(self.batch.terminated.cpu().numpy()[0])
        # only SectorCR truncates by itself (ownship left the sector, sector_cr_env.py:146)
        truncated = bool(self.batch.truncated.cpu().numpy()[0])
        return obs, reward, terminated, truncated, self._info()

    def render(self):
        if self.render_mode == "human":
            raise NotImplementedError("pygame rendering is out of scope of the MI355X step path")
        return None

    def close(self):
        self.batch.close()

    # conflict-detection outputs of the last step (StateBased, all pairs)
    def conflicts(self):
        if not self.batch.compute_cd:
            return None
        n = self.kind_cfg.num_ac
        cm = self.batch.conf_mask.cpu().numpy()[0].astype(np.uint64)
        return ((cm[:, None] >> np.arange(n, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)


def nan_if_zero(s, n):
    return s / n if n > 0 else math.nan
