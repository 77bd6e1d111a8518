"""WindFieldWrapper -- drop-in for bluesky_gym/wrappers/wind.py:8-66.

The reference wrapper adds the points to BlueSky's wind field after every reset
(``bs.traf.wind.addpointvne``, :28) -- every in-scope env's reset clears the field first
(``bs.traf.reset()``), so the field in force is always exactly these points -- and, with
``augment_obs``, appends ``wind_u`` / ``wind_v``: the wind at the ownship rotated into its
heading frame, divided by MAX_WIND (:56-66).  Here the field is handed to the device batch
once (``bsg_set_wind``); the kinematic effect (ActivePilot wind correction,
update_groundspeed, HDG command through the wind triangle) and the two observation terms
are computed inside the HIP step kernel.  ``WindFieldWrapper`` wraps a single env
(``gym.make``), ``VectorWindFieldWrapper`` a vector env (``gym.make_vec``).

Deviation: on the terminal step of VerticalCR / Descent / HorizontalCR the reference env
deletes its aircraft before the wrapper reads the ownship, so the reference raises
IndexError there; this build reports the wind at the terminal state instead.
"""
from __future__ import annotations

import numpy as np

from .. import _gym
from ..wind import WindTable

MAX_WIND = 50


class _WindMixin:
    def _setup(self, env, lat, lon, vnorth, veast, alt, augment_obs):
        self.lat = lat
        self.lon = lon
        self.vnorth = vnorth
        self.veast = veast
        self.alt = alt
        self.augment_obs = augment_obs
        if augment_obs:
            assert isinstance(env.observation_space, _gym.spaces.Dict), \
                "This wrapper only supports Dict observation spaces."
        target = env.unwrapped
        if not hasattr(target, "set_wind"):
            raise TypeError("WindFieldWrapper needs a bluesky_gym env (device batch)")
        target.set_wind(WindTable(lat, lon, vnorth, veast, alt), augment_obs=augment_obs)
        self.observation_space = target.observation_space
        if hasattr(target, "single_observation_space"):
            self.single_observation_space = target.single_observation_space


class WindFieldWrapper(_WindMixin, _gym.Wrapper):
    """Single env (gym.make)."""

    def __init__(self, env, lat, lon, vnorth, veast, alt=None, augment_obs=False):
        _gym.Wrapper.__init__(self, env)
        self._setup(env, lat, lon, vnorth, veast, alt, augment_obs)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def step(self, action):
        return self.env.step(action)


class VectorWindFieldWrapper(_WindMixin, _gym.VectorWrapper):
    """Vector env (gym.make_vec(..., vectorization_mode="vector_entry_point"))."""

    def __init__(self, env, lat, lon, vnorth, veast, alt=None, augment_obs=False):
        _gym.VectorWrapper.__init__(self, env)
        self._setup(env, lat, lon, vnorth, veast, alt, augment_obs)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def step(self, actions):
        return self.env.step(actions)
