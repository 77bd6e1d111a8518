"""VerticalCREnv-v0 -- drop-in for bluesky_gym/envs/vertical_cr_env.py (class
VerticalCREnv, :47).  NUM_INTRUDERS is 5 (redefined at vertical_cr_env.py:45)."""
from __future__ import annotations

from .. import config as cfgmod
from .. import spawn as spawnmod
from ._single import SingleEnvBase

DISTANCE_MARGIN = 5
NM2KM = 1.852
INTRUSION_PENALTY = -50
ALT_DIF_REWARD_SCALE = -5 / 3000
CRASH_PENALTY = -100
RWY_ALT_DIF_REWARD_SCALE = -50 / 3000
INTRUSION_DISTANCE = 5
VERTICAL_MARGIN = 1000 * 0.3048
ALT_MEAN, ALT_STD = 1500, 3000
VZ_MEAN, VZ_STD = 0, 5
RWY_DIS_MEAN, RWY_DIS_STD = 100, 200
DEFAULT_RWY_DIS = 200
RWY_LAT, RWY_LON = 52, 4
ACTION_2_MS = 12.5
ALT_MIN, ALT_MAX = 2000, 4000
TARGET_ALT_DIF = 500
AC_SPD = 150
ACTION_FREQUENCY = 30
NUM_INTRUDERS = 5


class VerticalCREnv(SingleEnvBase):
    """Vertical-speed control while descending to a runway, with intruders in conflict."""

    def __init__(self, render_mode=None, num_intruders=None, device=None, compute_cd=False):
        ni = NUM_INTRUDERS if num_intruders is None else num_intruders
        self._init_batch(cfgmod.vertical_config(ni, ACTION_FREQUENCY, 1.0, 0), render_mode,
                         device, compute_cd)
        self.num_intruders = ni

    def _spawn(self):
        return spawnmod.vertical_spawn(self.num_intruders)   # global np.random, reference order

    def _info(self):
        e = self.batch.envs
        return {"total_reward": float(e["total_reward"].cpu()[0]),
                "total_intrusions": int(e["total_intrusions"].cpu()[0]),
                "final_altitude": float(e["final_altitude"].cpu()[0])}
