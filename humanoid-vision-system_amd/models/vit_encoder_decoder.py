"""Drop-in alias of reference src/models/vit_encoder_decoder.py (implementation: hv_amd)."""
from hv_amd import PatchEmbedding, TransformerEncoderBlock, VisionTransformerEncoder, HybridVisionEncoder  # noqa: F401
