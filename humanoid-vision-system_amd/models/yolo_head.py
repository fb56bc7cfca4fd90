"""Drop-in alias of reference src/models/yolo_head.py (implementation: hv_amd)."""
from hv_amd import YOLOAnchorGenerator, YOLOPredictionHead, YOLODecoder, YOLOLoss, YOLODetectionHead  # noqa: F401
