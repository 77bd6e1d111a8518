"""MergeEnv-v0 -- drop-in for bluesky_gym/envs/merge_env.py (class MergeEnv, :48).

Module constants mirror merge_env.py:13-46; patching them before constructing an env
changes the env as it would the reference.  Live: NUM_AC, NUM_AC_STATE, ACTION_FREQUENCY,
AC_SPD (a whole number of m/s), D_HEADING, D_SPEED, INTRUSION_DISTANCE, DISTANCE_MARGIN,
REACH_REWARD, DRIFT_PENALTY, INTRUSION_PENALTY, SPAWN_DISTANCE_MIN/MAX and
INTRUDER_DISTANCE_MIN/MAX (the kernel's through bsg_set_params, the spawn draws through
spawn.merge_spawn).  Not live: NM2KM / MpS2Kt (unit constants), NUM_WAYPOINTS (unused by the
reference), RWY_* / FIX_* (the route is the kernel's configuration, config.RWY_LAT/FIX_LAT).
"""
from __future__ import annotations

import numpy as np

from .. import _native as nat
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
        params = {name: globals()[name] for name, _ in nat.MERGE_PARAMS}
        self._init_batch(cfgmod.merge_config(n, k, ACTION_FREQUENCY, 5.0, 0, ac_spd=AC_SPD,
                                             params=params), render_mode, device, compute_cd)
        self.nac = n
        self.wpt_lat, self.wpt_lon = FIX_LAT, FIX_LON
        self.rwy_lat, self.rwy_lon = RWY_LAT, RWY_LON

    def _spawn(self):
        # global `random`, reference order, this module's (patchable) constants
        return spawnmod.merge_spawn(self.nac, d_heading=D_HEADING,
                                    spawn_range=(SPAWN_DISTANCE_MIN, SPAWN_DISTANCE_MAX),
                                    intruder_range=(INTRUDER_DISTANCE_MIN, INTRUDER_DISTANCE_MAX))

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
