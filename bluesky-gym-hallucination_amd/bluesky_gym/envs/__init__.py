"""Env classes (bluesky_gym/envs/__init__.py:1-7 of the reference re-exports all)."""
from .descent_env import DescentEnv  # noqa: F401
from .merge_env import MergeEnv  # noqa: F401
from .vertical_cr_env import VerticalCREnv  # noqa: F401
from .horizontal_cr_env import HorizontalCREnv  # noqa: F401
from .sector_cr_env import SectorCREnv  # noqa: F401
from .static_obstacle_env import StaticObstacleEnv  # noqa: F401
from .plan_waypoint_env import PlanWaypointEnv  # noqa: F401
