"""Loss functions for YOLOv11 (MI355X-native), same public surface as the reference's losses/__init__.py."""

from .yolo_v8_loss import (  # noqa: F401
    v8DetectionLoss, BboxLoss, TaskAlignedAssigner,
    bbox_iou, bbox2dist, make_anchors, dist2bbox,
)

__all__ = [
    "v8DetectionLoss", "BboxLoss", "TaskAlignedAssigner",
    "bbox_iou", "bbox2dist", "make_anchors", "dist2bbox",
]
