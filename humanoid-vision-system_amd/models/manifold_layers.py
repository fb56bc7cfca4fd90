"""Drop-in alias of reference src/models/manifold_layers.py (implementation: hv_amd)."""
from hv_amd import SinkhornKnoppProjection, ManifoldHyperConnection, MultiHeadManifoldAttention, RMSNorm  # noqa: F401
