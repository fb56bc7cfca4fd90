"""Drop-in alias of reference src/models/feature_fusion.py (implementation: hv_amd)."""
from hv_amd import FeaturePyramidNetwork  # noqa: F401
