"""Drop-in alias of the reference's src/inference/engine.py."""
from hv_amd.engine import (AsyncInferenceEngine, InferenceConfig, InferenceEngine, StreamingPipeline,  # noqa: F401
                           preprocess_image)
