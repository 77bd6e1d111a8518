"""NoisyObservationWrapper -- drop-in for bluesky_gym/wrappers/uncertainty.py:4-31.

Adds N(0, noise_level) noise to every observation array, drawing from the global legacy
``np.random`` in the observation dict's key order like the reference.  For a device
vector env, ``step_tensors`` obs can be perturbed on the device instead
(``noisy_tensor``) with a torch generator; the NumPy path keeps the reference's RNG
consumption.
"""
from __future__ import annotations

import numpy as np

from .. import _gym


class NoisyObservationWrapper(_gym.Wrapper):
    def __init__(self, env, noise_level=0.1):
        super().__init__(env)
        self.noise_level = noise_level

    def reset(self, **kwargs):
        observation, info = self.env.reset(**kwargs)
        return self.add_noise(observation), info

    def step(self, action):
        observation, reward, done, truncated, info = self.env.step(action)
        return self.add_noise(observation), reward, done, truncated, info

    def add_noise(self, observation):
        if isinstance(observation, np.ndarray):
            return observation + np.random.normal(0, self.noise_level, size=observation.shape)
        if isinstance(observation, dict):
            return {key: (value + np.random.normal(0, self.noise_level, size=value.shape)
                          if isinstance(value, np.ndarray) else value)
                    for key, value in observation.items()}
        print('observation not an numpy array or dictionary, return observation unaltered')
        return observation

    def noisy_tensor(self, obs, generator=None):
        """Device-side variant for ``step_tensors`` rows (fp32 [E, obs_dim])."""
        import torch
        return obs + torch.randn(obs.shape, generator=generator, device=obs.device,
                                 dtype=obs.dtype) * self.noise_level
