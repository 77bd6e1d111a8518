"""Out of scope (see envs/_out_of_scope.py)."""
from ._out_of_scope import SectorCREnv  # noqa: F401
