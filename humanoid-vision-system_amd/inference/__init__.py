"""Drop-in alias of the reference's src/inference package (engine.py)."""
from hv_amd.engine import AsyncInferenceEngine, InferenceConfig, InferenceEngine  # noqa: F401
