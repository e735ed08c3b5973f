"""YOLOv11 models (MI355X-native), same public surface as the reference's models/__init__.py."""

from .yolo11_modules import (  # noqa: F401
    Conv, Bottleneck, C2f, C3k, C3k2, SPPF, Attention, PSA, C2PSA,
    DFL, Detect, Concat, make_anchors, dist2bbox,
)
from .yolo11_model import YOLOv11, build_yolo11  # noqa: F401

__all__ = [
    "Conv", "Bottleneck", "C2f", "C3k", "C3k2", "SPPF", "Attention", "PSA", "C2PSA",
    "DFL", "Detect", "Concat", "make_anchors", "dist2bbox",
    "YOLOv11", "build_yolo11",
]
