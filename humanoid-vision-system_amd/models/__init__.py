"""Drop-in for reference ``src/models`` (scripts do ``sys.path.insert(0, <pkg>)`` then
``from models.hybrid_vision import HybridVisionSystem``).  Everything is implemented in hv_amd."""
from hv_amd import *  # noqa: F401,F403
from hv_amd import (ConvMHCLayer, FeaturePyramidNetwork, HybridVisionBackbone, HybridVisionEncoder,  # noqa: F401
                    HybridVisionSystem, ManifoldHyperConnection, MultiHeadManifoldAttention, PatchEmbedding,
                    ResidualMHCLayer, RMSNorm, SinkhornKnoppProjection, TransformerEncoderBlock,
                    VisionTransformerEncoder, YOLOAnchorGenerator, YOLODecoder, YOLODetectionHead, YOLOLoss,
                    YOLOPredictionHead)
