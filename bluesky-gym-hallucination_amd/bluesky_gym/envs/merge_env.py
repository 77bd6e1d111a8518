"""MergeEnv-v0 -- drop-in for bluesky_gym/envs/merge_env.py (class MergeEnv, :48).

Module constants mirror merge_env.py:13-46; patching them (e.g. ``NUM_AC = 32``) before
constructing an env changes the env exactly as it would the reference.
"""
from __future__ import annotations

import numpy as np

from .. import config as cfgmod
from .. import spawn as spawnmod
from ._single import SingleEnvBase, nan_if_zero

DISTANCE_MARGIN = 10
REACH_REWARD = 1
DRIFT_PENALTY = -0.1
INTRUSION_PENALTY = -1
INTRUSION_DISTANCE = 4
SPAWN_DISTANCE_MIN = 50
SPAWN_DISTANCE_MAX = 200
INTRUDER_DISTANCE_MIN = 20
INTRUDER_DISTANCE_MAX = 500
D_HEADING = 15
D_SPEED = 20
AC_SPD = 100
NM2KM = 1.852
MpS2Kt = 1.94384
ACTION_FREQUENCY = 10
NUM_AC = 20
NUM_AC_STATE = 5
NUM_WAYPOINTS = 1
RWY_LAT = cfgmod.RWY_LAT
RWY_LON = cfgmod.RWY_LON
FIX_LAT, FIX_LON = cfgmod.FIX_LAT, cfgmod.FIX_LON


class MergeEnv(SingleEnvBase):
    """Single-agent arrival manager: the ownship merges into an NPC stream."""

    def __init__(self, render_mode=None, num_ac=None, num_ac_state=None, device=None,
                 compute_cd=False):
        n = NUM_AC if num_ac is None else num_ac
        k = NUM_AC_STATE if num_ac_state is None else num_ac_state
        self._init_batch(cfgmod.merge_config(n, k, ACTION_FREQUENCY, 5.0, 0), render_mode,
                         device, compute_cd)
        self.nac = n
        self.wpt_lat, self.wpt_lon = FIX_LAT, FIX_LON
        self.rwy_lat, self.rwy_lon = RWY_LAT, RWY_LON

    def _spawn(self):
        return spawnmod.merge_spawn(self.nac)          # global `random`, reference order

    def _info(self):
        e = self.batch.envs
        n = int(e["step_count"].cpu()[0])
        return {"total_reward": float(e["total_reward"].cpu()[0]),
                "faf_reach": int(e["faf_reached"].cpu()[0]),
                "average_drift": nan_if_zero(float(e["drift_sum"].cpu()[0]), n),
                "total_intrusions": int(e["total_intrusions"].cpu()[0])}

    @property
    def wpt_reach(self):
        return int(self.batch.envs["wpt_reach"].cpu()[0])
