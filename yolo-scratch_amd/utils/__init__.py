from .metrics import evaluate_detections, calculate_iou

__all__ = ["evaluate_detections", "calculate_iou"]
