"""SectorCREnv-v0 -- drop-in for bluesky_gym/envs/sector_cr_env.py (class SectorCREnv,
:40): a random sector polygon around the TU Delft AE faculty with a random number of
aircraft (density * area, at least 5); truncated when the ownship leaves the sector.
``num_ac`` is the aircraft capacity of the env (device lanes); an episode drawing more
raises (the reference has no cap, but more than 32 needs a density 3.5 sigma above its
mean)."""
from __future__ import annotations

from .. import areas
from .. import config as cfgmod
from ._single import SingleEnvBase, nan_if_zero

AC_DENSITY_RANGE = (0.003, 0.007)
AC_DENSITY_MU = 0.005
AC_DENSITY_SIGMA = 0.001
POLY_AREA_RANGE = (2400, 3750)
CENTER = areas.SECTOR_CENTER
ALTITUDE = 350
AC_SPD = 150
AC_TYPE = "A320"
ACTOR = "KL001"
NM2KM = 1.852
MpS2Kt = 1.94384
FL2M = 30.48
INTRUSION_DISTANCE = 5
ACTION_FREQUENCY = 5
NUM_AC_STATE = 4
DRIFT_PENALTY = -0.1
INTRUSION_PENALTY = -1
D_HEADING = 22.5
D_VELOCITY = 20 / 3


class SectorCREnv(SingleEnvBase):
    def __init__(self, render_mode=None, ac_density_mode="normal", num_ac=32, device=None,
                 compute_cd=False):
        self.density_mode = ac_density_mode
        self.capacity = num_ac
        self._init_batch(cfgmod.sector_config(num_ac, ACTION_FREQUENCY, 1.0, 0,
                                              "normal" if ac_density_mode == "normal" else "uniform"),
                         render_mode, device, compute_cd)

    def _spawn(self):
        return areas.sector_spawn(self.capacity, None,
                                  "normal" if self.density_mode == "normal" else "uniform")

    @property
    def num_ac(self):
        return int(self.batch.envs["env_geom"].cpu()[0, 0])

    def _info(self):
        e = self.batch.envs
        return {"total_reward": float(e["total_reward"].cpu()[0]),
                "total_intrusions": int(e["total_intrusions"].cpu()[0]),
                "average_drift": nan_if_zero(float(e["drift_sum"].cpu()[0]),
                                             int(e["step_count"].cpu()[0]))}
