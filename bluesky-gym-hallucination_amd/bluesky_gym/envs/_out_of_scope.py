"""Env ids the reference registers whose step path is outside this build's scope
(PlanWaypoint; not in SURVEY.md §8).  The ids
stay registered so ``register_envs()`` keeps the reference's id set; constructing one
raises with a pointer to DESIGN.md."""


class _OutOfScope:
    _ID = ""

    def __init__(self, *a, **k):
        raise NotImplementedError(
            f"{self._ID} is not provided by the MI355X step path (out of scope: "
            "see DESIGN.md §Scope); the other six env ids are.")


class PlanWaypointEnv(_OutOfScope):
    _ID = "PlanWaypointEnv-v0"
