"""Env wrappers of the reference (bluesky_gym/wrappers/): WindFieldWrapper (the wind path
runs inside the HIP step kernel) and NoisyObservationWrapper (host-side observation noise)."""
from .uncertainty import NoisyObservationWrapper  # noqa: F401
from .wind import VectorWindFieldWrapper, WindFieldWrapper  # noqa: F401
