from .metrics import calculate_ap, calculate_iou, calculate_iou_batch, evaluate_detections, evaluate_packed

__all__ = ["evaluate_detections", "evaluate_packed", "calculate_ap", "calculate_iou", "calculate_iou_batch"]
