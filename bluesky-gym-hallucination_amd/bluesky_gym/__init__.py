"""bluesky_gym -- MI355X-native vectorised BlueSky-Gym step path (drop-in API surface)."""
from ._native import BsgError  # noqa: F401
