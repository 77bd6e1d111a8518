"""Gymnasium API access.

Uses the real ``gymnasium`` when it is importable (the reference pins gymnasium==1.1.1,
pyproject.toml:11).  This image has no gymnasium, so a minimal stand-in with the same
names and semantics for the pieces this package uses is provided: ``Env``,
``spaces.Box``, ``spaces.Dict`` (sorted keys), ``register`` / ``make`` / ``make_vec`` /
``registry`` (incl. ``vector_entry_point``), ``TimeLimit``, ``Wrapper`` and
``vector.VectorEnv``.
It carries no simulation code.
"""
from __future__ import annotations

import importlib

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium is installed
    import gymnasium as gym  # noqa: F401
    from gymnasium import spaces  # noqa: F401
    from gymnasium.envs.registration import register, registry  # noqa: F401
    from gymnasium.vector import VectorEnv, VectorWrapper  # noqa: F401
    from gymnasium.wrappers import TimeLimit  # noqa: F401
    Env = gym.Env
    Wrapper = gym.Wrapper
    make = gym.make
    make_vec = gym.make_vec
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class _Space:
        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)
            return [seed]

        @property
        def np_random(self):
            if not hasattr(self, "_rng"):
                self._rng = np.random.default_rng()
            return self._rng

    class Box(_Space):
        def __init__(self, low, high, shape=None, dtype=np.float64):
            self.dtype = np.dtype(dtype)
            if shape is None:
                shape = np.shape(low) if np.ndim(low) else (1,)
            self.shape = tuple(shape)
            self.low = np.full(self.shape, low, self.dtype)
            self.high = np.full(self.shape, high, self.dtype)

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1e3)
            hi = np.where(np.isfinite(self.high), self.high, 1e3)
            return self.np_random.uniform(lo, hi, self.shape).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Dict(_Space):
        def __init__(self, spaces_=None, **kw):
            d = dict(spaces_ or {}, **kw)
            self.spaces = dict(sorted(d.items()))     # gymnasium sorts Dict keys

        def __getitem__(self, k):
            return self.spaces[k]

        def keys(self):
            return self.spaces.keys()

        def items(self):
            return self.spaces.items()

        def __iter__(self):
            return iter(self.spaces)

        def __len__(self):
            return len(self.spaces)

        def sample(self):
            return {k: s.sample() for k, s in self.spaces.items()}

        def contains(self, x):
            return set(x) == set(self.spaces) and all(self.spaces[k].contains(x[k]) for k in x)

    class _SpacesModule:
        Box = Box
        Dict = Dict

    spaces = _SpacesModule()

    class Env:
        metadata = {"render_modes": []}
        render_mode = None
        observation_space = None
        action_space = None

        def reset(self, *, seed=None, options=None):
            if seed is not None or not hasattr(self, "_np_random"):
                self._np_random = np.random.default_rng(seed)
            return None

        @property
        def np_random(self):
            if not hasattr(self, "_np_random"):
                self._np_random = np.random.default_rng()
            return self._np_random

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

    class Wrapper:
        """gymnasium.Wrapper: forwards reset/step/close; observation_space and
        action_space default to the wrapped env's unless assigned."""

        def __init__(self, env):
            self.env = env
            self._observation_space = None
            self._action_space = None

        @property
        def observation_space(self):
            return self._observation_space if self._observation_space is not None \
                else self.env.observation_space

        @observation_space.setter
        def observation_space(self, space):
            self._observation_space = space

        @property
        def action_space(self):
            return self._action_space if self._action_space is not None \
                else self.env.action_space

        @action_space.setter
        def action_space(self, space):
            self._action_space = space

        @property
        def unwrapped(self):
            return self.env.unwrapped

        def reset(self, **kw):
            return self.env.reset(**kw)

        def step(self, action):
            return self.env.step(action)

        def close(self):
            return self.env.close()

    class TimeLimit:
        """gymnasium.wrappers.TimeLimit: truncated once elapsed >= max_episode_steps."""

        def __init__(self, env, max_episode_steps):
            self.env = env
            self._max_episode_steps = max_episode_steps
            self._elapsed_steps = None

        def __getattr__(self, name):
            return getattr(self.env, name)

        @property
        def unwrapped(self):
            return self.env.unwrapped

        def reset(self, **kw):
            self._elapsed_steps = 0
            return self.env.reset(**kw)

        def step(self, action):
            obs, rew, term, trunc, info = self.env.step(action)
            self._elapsed_steps += 1
            if self._elapsed_steps >= self._max_episode_steps:
                trunc = True
            return obs, rew, term, trunc, info

    class VectorEnv:
        metadata = {"autoreset_mode": "NextStep"}
        num_envs = 1

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

    VectorWrapper = Wrapper

    class EnvSpec:
        def __init__(self, id, entry_point, max_episode_steps=None, vector_entry_point=None,
                     kwargs=None):
            self.id = id
            self.entry_point = entry_point
            self.max_episode_steps = max_episode_steps
            self.vector_entry_point = vector_entry_point
            self.kwargs = kwargs or {}

    registry = {}

    def register(id, entry_point=None, max_episode_steps=None, vector_entry_point=None,
                 kwargs=None, **_):
        registry[id] = EnvSpec(id, entry_point, max_episode_steps, vector_entry_point, kwargs)

    def _load(ep):
        mod, attr = ep.split(":")
        return getattr(importlib.import_module(mod), attr)

    def make(id, max_episode_steps=None, **kwargs):
        spec = registry[id]
        env = _load(spec.entry_point)(**{**spec.kwargs, **kwargs})
        steps = max_episode_steps if max_episode_steps is not None else spec.max_episode_steps
        return TimeLimit(env, steps) if steps else env

    def make_vec(id, num_envs=1, vectorization_mode="vector_entry_point", vector_kwargs=None,
                 **kwargs):
        spec = registry[id]
        if vectorization_mode != "vector_entry_point" or spec.vector_entry_point is None:
            raise NotImplementedError("only vectorization_mode='vector_entry_point' is "
                                      "available without gymnasium installed")
        kw = {**spec.kwargs, **kwargs, **(vector_kwargs or {})}
        kw.setdefault("max_episode_steps", spec.max_episode_steps)
        return _load(spec.vector_entry_point)(num_envs=num_envs, **kw)
