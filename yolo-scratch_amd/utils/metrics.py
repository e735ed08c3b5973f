"""Detection metrics: P / R / mAP50 / mAP50-95 on the MI355X (libyolomi ym_eval_detections).

Drop-in for /root/reference/yolo_scratch_cuda/utils/metrics.py: same functions, arguments
and return values --
  calculate_iou :19-46, calculate_iou_batch :49-81, evaluate_detections :84-274,
  calculate_ap :277-323.
evaluate_detections packs the per-image prediction / target dicts into flat device
arrays (image offsets, no per-box Python) and runs the whole evaluation -- conf filter,
per-image score sort, greedy matching at all IoU thresholds at once, the global
TP-before-FP score sort and the all-point AP -- as one chain of HIP launches
(csrc/metrics.hip); the host reads back 4 numbers.  CPU tensors are moved to the GPU;
there is no CPU fallback (the numpy restatement is oracle/metrics.py, test-only).
"""
from __future__ import annotations

from ctypes import c_double as ctypes_double
from typing import Dict, List, Sequence

import numpy as np
import torch

from yolomi._lib import YolomiError, call, lib, stream_ptr

GT_MAX_PER_IMAGE = 4096
_MAX_THR = 15


def _device(*tensors) -> torch.device:
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            return t.device
    if not torch.cuda.is_available():
        raise YolomiError("utils.metrics runs on the MI355X only: no GPU visible "
                          "(the CPU restatement lives in oracle/metrics.py and is test-only)")
    return torch.device("cuda", torch.cuda.current_device())


def _thresholds(iou_threshold: float) -> np.ndarray:
    """The reference's IoU thresholds (:131-136), fp64 exactly as np.arange makes them."""
    if iou_threshold == 0.5:
        return np.arange(0.5, 0.95 + 1e-6, 0.05)
    return np.arange(iou_threshold, min(1.0, iou_threshold + 0.45) + 1e-6, 0.05)


def evaluate_packed(pred_boxes: torch.Tensor, pred_scores: torch.Tensor, pred_counts: Sequence[int],
                    gt_boxes: torch.Tensor, gt_counts: Sequence[int], conf_threshold: float = 0.25,
                    iou_threshold: float = 0.5) -> Dict[str, object]:
    """evaluate_detections on flat device arrays: image b owns pred rows
    sum(pred_counts[:b]) .. +pred_counts[b] (xyxy fp32 + score) and GT rows likewise.

    Returns the reference's four metrics plus ``ap`` (one AP per IoU threshold),
    ``tp50`` / ``fp50`` and ``n_valid`` (predictions kept by ``conf_threshold``)."""
    dev = _device(pred_boxes, gt_boxes)
    n_img = len(pred_counts)
    if len(gt_counts) != n_img:
        raise YolomiError(f"evaluate: {n_img} prediction sets but {len(gt_counts)} target sets")
    max_gt = max(gt_counts) if n_img else 0
    if max_gt > GT_MAX_PER_IMAGE:
        raise YolomiError(f"evaluate: {max_gt} GT boxes in one image (the matcher holds {GT_MAX_PER_IMAGE})")
    thrs = _thresholds(float(iou_threshold))
    n_ap = len(thrs)
    if iou_threshold == 0.5:
        all_thr, pr_index = thrs, 0
    else:                                   # precision / recall are always counted at 0.5 (:252)
        all_thr, pr_index = np.concatenate([thrs, [0.5]]), n_ap
    n_thr = len(all_thr)
    if n_thr > _MAX_THR:
        raise YolomiError(f"evaluate: {n_thr} IoU thresholds (max {_MAX_THR})")
    pb = pred_boxes.to(dev, torch.float32).reshape(-1, 4).contiguous()
    ps = pred_scores.to(dev, torch.float32).reshape(-1).contiguous()
    gb = gt_boxes.to(dev, torch.float32).reshape(-1, 4).contiguous()
    n_pred, n_gt = pb.shape[0], gb.shape[0]
    if ps.numel() != n_pred or sum(pred_counts) != n_pred or sum(gt_counts) != n_gt:
        raise YolomiError("evaluate: counts do not match the packed arrays")
    offs = torch.tensor(np.concatenate([[0], np.cumsum(pred_counts, dtype=np.int64),
                                        [0], np.cumsum(gt_counts, dtype=np.int64)]).astype(np.int64))
    offs = offs.to(dev, non_blocking=True)
    poff, goff = offs[: n_img + 1], offs[n_img + 1:]
    ws_bytes = lib().ym_eval_workspace_size(n_img, max(n_pred, 1), n_thr)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    out = torch.empty(n_thr + 7, dtype=torch.float64, device=dev)
    thr_c = (ctypes_double * n_thr)(*[float(t) for t in all_thr])
    call("ym_eval_detections", pb.data_ptr(), ps.data_ptr(), poff.data_ptr(), gb.data_ptr(), goff.data_ptr(),
         n_img, n_pred, n_gt, max_gt, thr_c, n_thr, n_ap, pr_index, float(conf_threshold), ws.data_ptr(), ws_bytes,
         out.data_ptr(), stream_ptr(dev))
    o = out.cpu().tolist()                   # the single host sync
    r = o[n_thr:]
    if any(v != v for v in r[:4]):
        raise YolomiError("evaluate: an image exceeded the GT capacity of the matcher")
    return {"precision": r[0], "recall": r[1], "mAP50": r[2], "mAP50-95": r[3],
            "ap": o[:n_ap], "tp50": int(r[4]), "fp50": int(r[5]), "n_valid": int(r[6])}


def evaluate_detections(predictions: List[Dict], targets: List[Dict], conf_threshold: float = 0.25,
                        iou_threshold: float = 0.5) -> Dict[str, float]:
    """Reference :84-274.  predictions[i] = {boxes (N,4) xyxy, scores (N,), labels},
    targets[i] = {boxes (M,4), labels}; labels are ignored (class-agnostic, as the reference)."""
    n = min(len(predictions), len(targets))          # zip() semantics
    dev = _device(*[p["boxes"] for p in predictions[:n]], *[t["boxes"] for t in targets[:n]])
    pbs, pss, pc, gbs, gc = [], [], [], [], []
    for pred, tgt in zip(predictions[:n], targets[:n]):
        b = torch.as_tensor(pred["boxes"]).reshape(-1, 4)
        s = torch.as_tensor(pred["scores"]).reshape(-1)
        if len(b) == 0:
            s = s[:0]
        pbs.append(b.to(dev, torch.float32))
        pss.append(s.to(dev, torch.float32))
        pc.append(int(b.shape[0]))
        g = torch.as_tensor(tgt["boxes"]).reshape(-1, 4)
        gbs.append(g.to(dev, torch.float32))
        gc.append(int(g.shape[0]))
    empty4 = torch.zeros(0, 4, device=dev)
    pb = torch.cat(pbs) if pbs else empty4
    ps = torch.cat(pss) if pss else torch.zeros(0, device=dev)
    gb = torch.cat(gbs) if gbs else empty4
    r = evaluate_packed(pb, ps, pc, gb, gc, conf_threshold, iou_threshold)
    return {k: r[k] for k in ("precision", "recall", "mAP50", "mAP50-95")}


def calculate_ap(tp: List[float], fp: List[float], n_gt: int) -> float:
    """Reference :277-323: all-point AP of TP / FP score lists (ym_eval_ap)."""
    dev = _device()
    scores = torch.tensor(list(tp) + list(fp), dtype=torch.float32).to(dev)
    flags = torch.tensor([1] * len(tp) + [0] * len(fp), dtype=torch.uint8).to(dev)
    n = scores.numel()
    ws_bytes = lib().ym_eval_workspace_size(1, max(n, 1), 1)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    out = torch.empty(8, dtype=torch.float64, device=dev)
    call("ym_eval_ap", scores.data_ptr(), flags.data_ptr(), n, int(n_gt), ws.data_ptr(), ws_bytes, out.data_ptr(),
         stream_ptr(dev))
    return float(out[0].item())


def calculate_iou_batch(boxes1: torch.Tensor, boxes2: torch.Tensor) -> torch.Tensor:
    """Reference :49-81: (N, M) IoU of xyxy boxes, fp32 (ym_iou_matrix)."""
    dev = _device(boxes1, boxes2)
    a = torch.as_tensor(boxes1).to(dev, torch.float32).reshape(-1, 4).contiguous()
    b = torch.as_tensor(boxes2).to(dev, torch.float32).reshape(-1, 4).contiguous()
    out = torch.empty(a.shape[0], b.shape[0], dtype=torch.float32, device=dev)
    call("ym_iou_matrix", a.data_ptr(), b.data_ptr(), a.shape[0], b.shape[0], out.data_ptr(), stream_ptr(dev))
    return out


def calculate_iou(box1, box2):
    """Reference :19-46: IoU of two xyxy boxes (0-d tensor), 0.0 when the union is not positive.
    Four scalars: evaluated with device tensor ops in the reference's order (bare union, no eps)."""
    dev = _device(box1, box2)
    b1 = torch.as_tensor(box1).to(dev, torch.float32).reshape(4)
    b2 = torch.as_tensor(box2).to(dev, torch.float32).reshape(4)
    inter = (torch.clamp(torch.min(b1[2], b2[2]) - torch.max(b1[0], b2[0]), min=0.0)
             * torch.clamp(torch.min(b1[3], b2[3]) - torch.max(b1[1], b2[1]), min=0.0))
    union = (b1[2] - b1[0]) * (b1[3] - b1[1]) + (b2[2] - b2[0]) * (b2[3] - b2[1]) - inter
    if union <= 0:
        return 0.0
    return inter / union
