"""TEST ORACLE ONLY (imported by tests/, smoke() and bench.py's cpu_baseline leg).

CPU restatement of the detection metrics: P / R / mAP50 / mAP50-95 (class-agnostic
greedy matching), numpy, with the semantics of
/root/reference/yolo_scratch_cuda/utils/metrics.py:
  calculate_iou :19-46, calculate_iou_batch :49-81, evaluate_detections
  :84-274 (conf filter `>=`, score-sorted greedy match to the best unmatched
  GT, labels ignored, thresholds 0.5:0.05:0.95), calculate_ap :277-323
  (all-point interpolation).
Pinned by tests/golden/metrics.npz (the reference's own evaluate_detections run on
the committed inputs, tests/golden/gen_golden.py:gen_metrics).  The product path is
utils/metrics.py -> libyolomi ym_eval_detections (csrc/metrics.hip).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch


def calculate_iou(box1, box2):
    b1 = torch.as_tensor(box1, dtype=torch.float32)
    b2 = torch.as_tensor(box2, dtype=torch.float32)
    iw = torch.clamp(torch.min(b1[2], b2[2]) - torch.max(b1[0], b2[0]), min=0.0)
    ih = torch.clamp(torch.min(b1[3], b2[3]) - torch.max(b1[1], b2[1]), min=0.0)
    inter = iw * ih
    union = (b1[2] - b1[0]) * (b1[3] - b1[1]) + (b2[2] - b2[0]) * (b2[3] - b2[1]) - inter
    if union <= 0:
        return 0.0
    return inter / union


def calculate_iou_batch(boxes1, boxes2):
    a = np.asarray(boxes1, np.float32)[:, None, :]
    b = np.asarray(boxes2, np.float32)[None, :, :]
    iw = np.clip(np.minimum(a[..., 2], b[..., 2]) - np.maximum(a[..., 0], b[..., 0]), 0.0, None)
    ih = np.clip(np.minimum(a[..., 3], b[..., 3]) - np.maximum(a[..., 1], b[..., 1]), 0.0, None)
    inter = iw * ih
    area_a = (a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1])
    area_b = (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
    union = area_a + area_b - inter
    return inter / (union + np.float32(1e-6))


def calculate_ap(tp: List[float], fp: List[float], n_gt: int) -> float:
    if n_gt == 0:
        return 0.0
    dets = sorted([(s, 1) for s in tp] + [(s, 0) for s in fp], key=lambda x: x[0], reverse=True)
    if not dets:
        return 0.0
    flags = np.asarray([d[1] for d in dets])
    tpc = np.cumsum(flags)
    fpc = np.cumsum(1 - flags)
    prec = tpc / (tpc + fpc + 1e-6)
    rec = tpc / n_gt
    mrec = np.concatenate([[0.0], rec, [1.0]])
    mpre = np.concatenate([[0.0], prec, [0.0]])
    mpre = np.maximum.accumulate(mpre[::-1])[::-1]
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return float(np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1]))


def _match(iou: np.ndarray, thr: float) -> np.ndarray:
    """Greedy: each prediction (score order) takes the best unmatched GT; TP if IoU >= thr."""
    n_pred, n_gt = iou.shape
    used = np.zeros(n_gt, bool)
    tp = np.zeros(n_pred, bool)
    for i in range(n_pred):
        if used.all():
            continue
        row = np.where(used, -np.inf, iou[i])
        j = int(np.argmax(row))
        if row[j] >= thr:
            tp[i] = True
            used[j] = True
    return tp


def thresholds(iou_threshold: float) -> np.ndarray:
    """evaluate_detections' IoU thresholds (utils/metrics.py:131-136)."""
    if iou_threshold == 0.5:
        return np.arange(0.5, 0.95 + 1e-6, 0.05)
    return np.arange(iou_threshold, min(1.0, iou_threshold + 0.45) + 1e-6, 0.05)


def evaluate_detections(predictions: List[Dict], targets: List[Dict], conf_threshold: float = 0.25,
                        iou_threshold: float = 0.5, per_threshold: bool = False) -> Dict[str, float]:
    thrs = thresholds(iou_threshold)
    tps = [[] for _ in thrs]
    fps = [[] for _ in thrs]
    tp50, fp50, n_gt = 0, 0, 0
    for pred, tgt in zip(predictions, targets):
        pb = np.asarray(torch.as_tensor(pred["boxes"]).cpu(), np.float32).reshape(-1, 4)
        ps = np.asarray(torch.as_tensor(pred["scores"]).cpu(), np.float32).reshape(-1)
        if len(pb):
            keep = ps >= np.float32(conf_threshold)
            pb, ps = pb[keep], ps[keep]
        tb = np.asarray(torch.as_tensor(tgt["boxes"]).cpu(), np.float32).reshape(-1, 4)
        n_gt += len(tb)
        if len(pb) == 0:
            continue
        if len(tb) == 0:
            for k in range(len(thrs)):
                fps[k].extend(ps.tolist())
            fp50 += len(ps)
            continue
        order = np.argsort(-ps, kind="stable")
        pb, ps = pb[order], ps[order]
        iou = calculate_iou_batch(pb, tb)
        for k, t in enumerate(thrs):
            tp = _match(iou, t)
            tps[k].extend(ps[tp].tolist())
            fps[k].extend(ps[~tp].tolist())
        tp = _match(iou, 0.5)
        tp50 += int(tp.sum())
        fp50 += int((~tp).sum())
    aps = [calculate_ap(tps[k], fps[k], n_gt) for k in range(len(thrs))]
    precision = tp50 / (tp50 + fp50) if (tp50 + fp50) > 0 else 0.0
    recall = tp50 / n_gt if n_gt > 0 else 0.0
    out = {"precision": precision, "recall": recall, "mAP50": aps[0] if aps else 0.0,
           "mAP50-95": float(np.mean(aps)) if aps else 0.0}
    if per_threshold:
        out.update(ap=aps, tp50=tp50, fp50=fp50)
    return out
