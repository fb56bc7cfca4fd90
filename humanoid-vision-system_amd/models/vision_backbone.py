"""Drop-in alias of reference src/models/vision_backbone.py (implementation: hv_amd)."""
from hv_amd import ConvMHCLayer, ResidualMHCLayer, HybridVisionBackbone  # noqa: F401
