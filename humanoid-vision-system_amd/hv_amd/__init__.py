"""hv_amd -- MI355X-native HybridVision hot path (HIP kernels behind the reference nn.Module API).

The classes mirror reference src/models (names, constructor signatures, parameter and buffer
names/shapes) so reference checkpoints and call sites keep working; their forward passes run
on hand-written gfx950 kernels in libhvs.so (see include/hv_kernels.h).
"""
from .manifold import (ManifoldHyperConnection, MultiHeadManifoldAttention, RMSNorm,  # noqa: F401
                       SinkhornKnoppProjection)
from .backbone import ConvMHCLayer, HybridVisionBackbone, ResidualMHCLayer  # noqa: F401
from .vit import (HybridVisionEncoder, PatchEmbedding, TransformerEncoderBlock,  # noqa: F401
                  VisionTransformerEncoder)
from .detect import (FeaturePyramidNetwork, HybridVisionSystem, YOLOAnchorGenerator,  # noqa: F401
                     YOLODecoder, YOLODetectionHead, YOLOLoss, YOLOPredictionHead)
from . import library  # noqa: F401,E402  (registers the torch.ops.hv.* dispatcher operators)

__version__ = "0.1.0"
