"""Drop-in alias of reference src/models/hybrid_vision.py (implementation: hv_amd)."""
from hv_amd import HybridVisionSystem  # noqa: F401
