"""DescentEnv-v0 -- drop-in for bluesky_gym/envs/descent_env.py (class DescentEnv, :32)."""
from __future__ import annotations

from .. import config as cfgmod
from .. import spawn as spawnmod
from ._single import SingleEnvBase

ALT_MEAN, ALT_STD = 1500, 3000
VZ_MEAN, VZ_STD = 0, 5
RWY_DIS_MEAN, RWY_DIS_STD = 100, 200
ACTION_2_MS = 12.5
ALT_DIF_REWARD_SCALE = -5 / 3000
CRASH_PENALTY = -100
RWY_ALT_DIF_REWARD_SCALE = -50 / 3000
ALT_MIN, ALT_MAX = 2000, 4000
TARGET_ALT_DIF = 500
AC_SPD = 150
ACTION_FREQUENCY = 30


class DescentEnv(SingleEnvBase):
    """Climb / descend to a target altitude, then descend before the runway."""

    def __init__(self, render_mode=None, device=None):
        self._init_batch(cfgmod.descent_config(ACTION_FREQUENCY, 1.0, 0), render_mode, device, False)

    def _spawn(self):
        return spawnmod.descent_spawn()                      # global np.random, reference order

    def _info(self):
        e = self.batch.envs
        return {"total_reward": float(e["total_reward"].cpu()[0]),
                "final_altitude": float(e["final_altitude"].cpu()[0])}
