"""Env ids the reference registers whose step path is outside this build's scope
(HorizontalCR, SectorCR, StaticObstacle, PlanWaypoint).  The ids
stay registered so ``register_envs()`` keeps the reference's id set; constructing one
raises with a pointer to DESIGN.md."""


class _OutOfScope:
    _ID = ""

    def __init__(self, *a, **k):
        raise NotImplementedError(
            f"{self._ID} is not provided by the MI355X step path (out of scope: "
            "see DESIGN.md §Scope); MergeEnv-v0, VerticalCREnv-v0 and DescentEnv-v0 are.")


class HorizontalCREnv(_OutOfScope):
    _ID = "HorizontalCREnv-v0"


class SectorCREnv(_OutOfScope):
    _ID = "SectorCREnv-v0"


class StaticObstacleEnv(_OutOfScope):
    _ID = "StaticObstacleEnv-v0"


class PlanWaypointEnv(_OutOfScope):
    _ID = "PlanWaypointEnv-v0"
