"""Drop-in alias of the reference's src/inference/engine.py."""
from hv_amd.engine import AsyncInferenceEngine, InferenceConfig, InferenceEngine, preprocess_image  # noqa: F401
