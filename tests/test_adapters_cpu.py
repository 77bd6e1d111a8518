"""Host side of the learner adapters (no GPU): the SB3 and RLlib adapters import without
their libraries and cover every id register_envs() registers with a vector entry point."""
import bluesky_gym
from bluesky_gym import _gym


def test_adapters_cover_every_registered_id():
    from bluesky_gym.rllib import RLlibVectorEnv
    from bluesky_gym.sb3 import VECTOR_ENVS, SB3VecEnv
    bluesky_gym.register_envs()
    ids = {"MergeEnv-v0", "VerticalCREnv-v0", "DescentEnv-v0", "HorizontalCREnv-v0",
           "StaticObstacleEnv-v0", "SectorCREnv-v0", "PlanWaypointEnv-v0"}
    assert set(VECTOR_ENVS) == ids
    for env_id, cls in VECTOR_ENVS.items():
        spec = _gym.registry[env_id] if hasattr(_gym, "registry") else None
        if spec is not None and getattr(spec, "vector_entry_point", None):
            assert spec.vector_entry_point.endswith(":" + cls.__name__)
    for api in ("vector_reset", "reset_at", "restart_at", "vector_step", "get_sub_environments"):
        assert callable(getattr(RLlibVectorEnv, api))
    for api in ("reset", "step_async", "step_wait", "env_is_wrapped", "get_attr"):
        assert callable(getattr(SB3VecEnv, api))
