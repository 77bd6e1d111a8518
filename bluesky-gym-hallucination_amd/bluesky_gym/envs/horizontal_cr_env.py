"""HorizontalCREnv-v0 -- drop-in for bluesky_gym/envs/horizontal_cr_env.py (class
HorizontalCREnv, :32): heading control towards a waypoint 100-150 km north with NUM_INTRUDERS
level intruders placed in conflict by creconfs."""
from __future__ import annotations

from .. import config as cfgmod
from .. import spawn as spawnmod
from ._single import SingleEnvBase, nan_if_zero

DISTANCE_MARGIN = 5
REACH_REWARD = 1
DRIFT_PENALTY = -0.1
INTRUSION_PENALTY = -1
NUM_INTRUDERS = 5
NUM_WAYPOINTS = 1
INTRUSION_DISTANCE = 5
WAYPOINT_DISTANCE_MIN = 100
WAYPOINT_DISTANCE_MAX = 150
D_HEADING = 45
AC_SPD = 150
NM2KM = 1.852
ACTION_FREQUENCY = 10


class HorizontalCREnv(SingleEnvBase):
    """Horizontal conflict resolution: reach the waypoint while avoiding intruders."""

    def __init__(self, render_mode=None, num_intruders=None, device=None, compute_cd=False):
        ni = NUM_INTRUDERS if num_intruders is None else num_intruders
        self._init_batch(cfgmod.horizontal_config(ni, ACTION_FREQUENCY, 5.0, 0), render_mode,
                         device, compute_cd)
        self.num_intruders = ni

    def _spawn(self):
        return spawnmod.horizontal_spawn(self.num_intruders)   # global np.random, reference order

    @property
    def wpt_lat(self):
        return [float(self.batch.envs["env_wpt_lat"].cpu()[0])]

    @property
    def wpt_lon(self):
        return [float(self.batch.envs["env_wpt_lon"].cpu()[0])]

    def _info(self):
        e = self.batch.envs
        return {"total_reward": float(e["total_reward"].cpu()[0]),
                "total_intrusions": int(e["total_intrusions"].cpu()[0]),
                "average_drift": nan_if_zero(float(e["drift_sum"].cpu()[0]),
                                             int(e["step_count"].cpu()[0]))}
