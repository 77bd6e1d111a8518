"""StaticObstacleEnv-v0 -- drop-in for bluesky_gym/envs/static_obstacle_env.py (class
StaticObstacleEnv, :43): fly to a waypoint 100-170 km away around NUM_OBSTACLES random
restricted-area polygons; the reward is evaluated after every substep (:132-150)."""
from __future__ import annotations

from .. import areas
from .. import config as cfgmod
from ._single import SingleEnvBase, nan_if_zero

DISTANCE_MARGIN = 5
REACH_REWARD = 1
DRIFT_PENALTY = -0.01
RESTRICTED_AREA_INTRUSION_PENALTY = -5
INTRUSION_DISTANCE = 5
WAYPOINT_DISTANCE_MIN = 100
WAYPOINT_DISTANCE_MAX = 170
OBSTACLE_DISTANCE_MIN = 20
OBSTACLE_DISTANCE_MAX = 150
D_HEADING = 45
D_SPEED = 20 / 3
AC_SPD = 150
ALTITUDE = 350
NM2KM = 1.852
MpS2Kt = 1.94384
ACTION_FREQUENCY = 10
NUM_OBSTACLES = 10
NUM_WAYPOINTS = 1
OBSTACLE_AREA_RANGE = (50, 1000)
CENTER = (51.990426702297746, 4.376124857109851)


class StaticObstacleEnv(SingleEnvBase):
    def __init__(self, render_mode=None, device=None):
        self._init_batch(cfgmod.static_config(ACTION_FREQUENCY, 1.0, 0), render_mode, device,
                         False)

    def _spawn(self):
        return areas.static_spawn()          # global np.random, reference order

    def _info(self):
        e = self.batch.envs
        aux = e["env_aux"].cpu().numpy()[0]
        return {"total_reward": float(e["total_reward"].cpu()[0]),
                "waypoint_reached": int(e["wpt_reach"].cpu()[0]),
                "crashed": int(aux[3]),
                "average_drift": nan_if_zero(float(e["drift_sum"].cpu()[0]), int(aux[2]))}
