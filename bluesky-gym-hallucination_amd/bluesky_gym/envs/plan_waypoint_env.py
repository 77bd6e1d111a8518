"""PlanWaypointEnv-v0 -- drop-in for bluesky_gym/envs/plan_waypoint_env.py (class
PlanWaypointEnv, :25).

Fly over as many of five waypoints as possible (heading actions only).  As in the
reference, reset() does not clear the traffic: after a truncation (TimeLimit) the next
episode starts from where the aircraft is, with new waypoints drawn around it; a
terminated episode (all five reached) deletes the aircraft, so the next one starts at
52N 4E again (plan_waypoint_env.py:156-171, 189-193).
"""
from __future__ import annotations

from .. import config as cfgmod
from .. import spawn as spawnmod
from ._single import SingleEnvBase

DISTANCE_MARGIN = 5
WAYPOINT_DISTANCE_MIN = 0
WAYPOINT_DISTANCE_MAX = 75
NUM_WAYPOINTS = 5
REACH_REWARD = 1
AC_SPD = 150
D_HEADING = 45
ACTION_FREQUENCY = 10


class PlanWaypointEnv(SingleEnvBase):
    """Waypoint collection with heading control (plan_waypoint_env.py)."""

    def __init__(self, render_mode=None, device=None):
        self._init_batch(cfgmod.plan_waypoint_config(ACTION_FREQUENCY, 1.0, 0), render_mode,
                         device, False)

    def _spawn(self):
        return spawnmod.plan_spawn()                         # global np.random, reference order

    def _info(self):
        e = self.batch.envs
        wr = int(e["wpt_reach"].cpu()[0])
        return {"total_reward": float(e["total_reward"].cpu()[0]),
                "waypoints_completed": bin(wr).count("1")}
