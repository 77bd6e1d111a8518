"""bluesky_gym -- MI355X-native vectorised BlueSky-Gym step path.

Drop-in for the reference package's public surface (bluesky_gym/__init__.py:4-46):
``register_envs()`` registers the same seven ids with the same entry points and
TimeLimit lengths, and adds a ``vector_entry_point`` to each (every step path runs on
the GPU), so ``gym.make_vec(id, num_envs, vectorization_mode="vector_entry_point")``
returns one device-resident batch.  SB3 is imported lazily (bluesky_gym.sb3).
"""
from ._native import BsgError  # noqa: F401
from . import _gym

__all__ = ["register_envs", "BsgError"]


def register_envs():
    """Import the envs module so that environments / scenarios register themselves."""
    reg = _gym.register
    reg(id="DescentEnv-v0", entry_point="bluesky_gym.envs.descent_env:DescentEnv",
        max_episode_steps=300, vector_entry_point="bluesky_gym.vector:DescentVectorEnv")
    reg(id="PlanWaypointEnv-v0", entry_point="bluesky_gym.envs.plan_waypoint_env:PlanWaypointEnv",
        max_episode_steps=300, vector_entry_point="bluesky_gym.vector:PlanWaypointVectorEnv")
    reg(id="HorizontalCREnv-v0", entry_point="bluesky_gym.envs.horizontal_cr_env:HorizontalCREnv",
        max_episode_steps=300, vector_entry_point="bluesky_gym.vector:HorizontalCRVectorEnv")
    reg(id="VerticalCREnv-v0", entry_point="bluesky_gym.envs.vertical_cr_env:VerticalCREnv",
        max_episode_steps=300, vector_entry_point="bluesky_gym.vector:VerticalCRVectorEnv")
    reg(id="SectorCREnv-v0", entry_point="bluesky_gym.envs.sector_cr_env:SectorCREnv",
        max_episode_steps=200, vector_entry_point="bluesky_gym.vector:SectorCRVectorEnv")
    reg(id="StaticObstacleEnv-v0",
        entry_point="bluesky_gym.envs.static_obstacle_env:StaticObstacleEnv",
        max_episode_steps=100, vector_entry_point="bluesky_gym.vector:StaticObstacleVectorEnv")
    reg(id="MergeEnv-v0", entry_point="bluesky_gym.envs.merge_env:MergeEnv",
        max_episode_steps=50, vector_entry_point="bluesky_gym.vector:MergeVectorEnv")
