"""RLlib adapter (the reference README's second consumer, README.md:36: "algorithms from
standardized libraries such as Stable-Baselines3 or RLlib").

RLlib's new API stack consumes a Gymnasium ``VectorEnv`` directly; ``gym.make_vec(id,
num_envs, vectorization_mode="vector_entry_point")`` (bluesky_gym.vector) is one, with
Gymnasium 1.x's NEXT_STEP autoreset.  ``RLlibVectorEnv`` serves the legacy stack's
``ray.rllib.env.vector_env.VectorEnv`` contract: ``vector_reset`` / ``vector_step``
return per-env lists, the env runner calls ``reset_at(i)`` for every env that finished.
The batch runs SAME_STEP autoreset, so a finished env was already respawned inside the
step launch: ``vector_step`` reports its terminal observation (``final_obs``) and
``reset_at`` hands out the stored reset observation without another launch.  Ray is
not required to import this module; when it is installed the class subclasses
``ray.rllib.env.vector_env.VectorEnv``.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native as nat
from .sb3 import VECTOR_ENVS, episode_infos
from .vector import BlueSkyVectorEnv

try:  # pragma: no cover
    from ray.rllib.env.vector_env import VectorEnv as _RLlibBase
except ImportError:
    _RLlibBase = object


class RLlibVectorEnv(_RLlibBase):
    def __init__(self, env_id: str, num_envs: int, *, seed=0, device=None, **env_kwargs):
        self.venv: BlueSkyVectorEnv = VECTOR_ENVS[env_id](
            num_envs=num_envs, seed=seed, device=device, autoreset=nat.AUTORESET_SAME_STEP,
            **env_kwargs)
        self.num_envs = num_envs
        self.observation_space = self.venv.single_observation_space
        self.action_space = self.venv.single_action_space
        self._reset_obs = {}       # env index -> reset obs of an env respawned in vector_step

    def _rows(self, flat):
        """[E, O] fp32 rows -> per-env Dict observations (float64, sorted keys)."""
        parts = self.venv.layout.split(flat)
        return [{k: v[i] for k, v in parts.items()} for i in range(flat.shape[0])]

    # ------------------------------------------------------------- RLlib VectorEnv API
    def vector_reset(self, *, seeds=None, options=None):
        """All envs from a fresh episode; seeds[0] (if given) reseeds the batch."""
        seed = None if not seeds else seeds[0]
        obs, info = self.venv.reset(seed=seed)
        self._reset_obs.clear()
        per = [{k: v[i] for k, v in obs.items()} for i in range(self.num_envs)]
        return per, [self._info(info, i) for i in range(self.num_envs)]

    def reset_at(self, index=None, *, seed=None, options=None):
        """A finished env's new episode (already spawned by the step that ended it); any
        other env is reset now by a masked reset launch."""
        i = 0 if index is None else int(index)
        if seed is None and i in self._reset_obs:
            return self._reset_obs.pop(i), {}
        b = self.venv.batch
        m = torch.zeros(self.num_envs, dtype=torch.uint8, device=b.device)
        m[i] = 1
        b.reset(env_mask=m)
        self._reset_obs.pop(i, None)
        return self._rows(b.obs[i:i + 1].cpu().numpy())[0], {}

    def restart_at(self, index=None):
        self.reset_at(index)

    def vector_step(self, actions):
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions, np.float64))
        b = self.venv.batch
        obs_t, rew_t, term_t, trunc_t = self.venv.step_tensors(a)
        term = term_t.cpu().numpy().astype(bool)
        trunc = trunc_t.cpu().numpy().astype(bool)
        done = term | trunc
        obs = self._rows(obs_t.cpu().numpy())
        if done.any():
            fin = self._rows(b.final_obs.cpu().numpy())
            for i in np.nonzero(done)[0]:
                self._reset_obs[int(i)] = obs[i]
                obs[i] = fin[i]
        return (obs, rew_t.cpu().numpy().astype(np.float64).tolist(), term.tolist(),
                trunc.tolist(), episode_infos(self.venv, done, term, trunc))

    def get_sub_environments(self):
        return []

    def try_render_at(self, index=None):
        return None

    def close(self):
        self.venv.close()

    @staticmethod
    def _info(info, i):
        return {k: (v[i].item() if hasattr(v[i], "item") else v[i])
                for k, v in info.items() if not k.startswith("_")}
