"""Decode + NMS postprocess on the GPU (libyolomi ym_decode_nms / ym_nms / ym_iou_row).

Host-side mirror of decode_predictions_for_metrics / nms_simple /
calculate_iou_batch_simple (reference train_yolo11_cuda.py:265-437): same
arguments, same return types.  The whole batch is one pair of launches; the
host synchronises once (the per-image counts) instead of once per kept box.
"""
from __future__ import annotations

import torch

from ._lib import call, ptr, require_device, stream_ptr


def iou_row(box1: torch.Tensor, boxes2: torch.Tensor) -> torch.Tensor:
    require_device(box1, boxes2)
    b1 = box1.reshape(4).float().contiguous()
    b2 = boxes2.float().contiguous()
    out = torch.empty(b2.shape[0], device=b2.device, dtype=torch.float32)
    call("ym_iou_row", ptr(b1), ptr(b2), b2.shape[0], ptr(out), stream_ptr(b2.device))
    return out


def nms(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float) -> torch.Tensor:
    """Keep indices (int64, device) in kept order."""
    require_device(boxes, scores)
    from ._lib import lib
    n = boxes.shape[0]
    b = boxes.float().contiguous()
    s = scores.float().contiguous()
    ws_bytes = lib().ym_nms_workspace_size(1, max(n, 1))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=b.device)
    keep = torch.empty(max(n, 1), dtype=torch.int64, device=b.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=b.device)
    call("ym_nms", ptr(b), ptr(s), n, float(iou_threshold), ptr(ws), ws_bytes, ptr(keep), ptr(cnt),
         stream_ptr(b.device))
    return keep[: int(cnt.item())]


def decode_nms(pred: torch.Tensor, img_size, conf: float, iou_thr: float):
    """Batched decode+NMS of pred read as (B, N, 4+C).  Returns per-image dicts."""
    require_device(pred)
    from ._lib import lib
    p = pred.float()
    if p.stride(-1) < 1:
        p = p.contiguous()
    B, N, W = p.shape
    C = W - 4
    dev = p.device
    ws_bytes = lib().ym_nms_workspace_size(B, max(N, 1))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    cnt = torch.empty(B, dtype=torch.int32, device=dev)          # every count is written by the launch
    boxes = torch.empty(B, N, 4, dtype=torch.float32, device=dev)
    scores = torch.empty(B, N, dtype=torch.float32, device=dev)
    labels = torch.empty(B, N, dtype=torch.int64, device=dev)
    index = torch.empty(B, N, dtype=torch.int64, device=dev)
    # a row's elements may be strided (the anchor-major view y.transpose(1, 2) of the eval output): read in place
    call("ym_decode_nms_strided", ptr(p), B, N, C, p.stride(1), p.stride(0), p.stride(2), float(conf), float(iou_thr),
         float(img_size), ptr(ws), ws_bytes, ptr(cnt), ptr(boxes), ptr(scores), ptr(labels), ptr(index),
         stream_ptr(dev))
    counts = cnt.cpu().tolist()                      # the single host sync of the batch
    return [{"boxes": boxes[b, :k], "scores": scores[b, :k], "labels": labels[b, :k]} for b, k in enumerate(counts)]
