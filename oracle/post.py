"""Decode + NMS oracle (numpy fp32 + nms_ref.c) — TEST ORACLE ONLY.

Restates decode_predictions_for_metrics / nms_simple / calculate_iou_batch_simple
(/root/reference/yolo_scratch_cuda/train_yolo11_cuda.py:265-437).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        so = _HERE / "libnms_oracle.so"
        if not so.exists():
            subprocess.run(["make", "-C", str(_HERE)], check=True, capture_output=True)
        L = ctypes.CDLL(str(so))
        L.oracle_nms.restype = ctypes.c_int64
        L.oracle_nms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p]
        L.oracle_iou_row.restype = None
        L.oracle_iou_row.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        _LIB = L
    return _LIB


def nms(boxes: np.ndarray, scores: np.ndarray, thr: float) -> np.ndarray:
    boxes = np.ascontiguousarray(boxes, np.float32)
    scores = np.ascontiguousarray(scores, np.float32)
    n = len(scores)
    keep = np.zeros(max(n, 1), np.int64)
    k = lib().oracle_nms(boxes.ctypes.data, scores.ctypes.data, n, ctypes.c_float(np.float32(thr)), keep.ctypes.data)
    return keep[:k]


def iou_row(b1: np.ndarray, b2: np.ndarray) -> np.ndarray:
    b1 = np.ascontiguousarray(b1, np.float32).reshape(4)
    b2 = np.ascontiguousarray(b2, np.float32)
    out = np.zeros(len(b2), np.float32)
    lib().oracle_iou_row(b1.ctypes.data, b2.ctypes.data, len(b2), out.ctypes.data)
    return out


def decode(pred: np.ndarray, img_size: int, conf: float, iou_thr: float):
    """decode_predictions_for_metrics (train_yolo11_cuda.py:265-358); pred read as (B, N, 4+C)."""
    pred = np.asarray(pred, np.float32)
    outs = []
    for b in range(pred.shape[0]):
        p = pred[b]
        cls = p[:, 4:]
        mx = cls.max(1)
        lab = cls.argmax(1)
        m = mx > np.float32(conf)
        if not m.any():
            outs.append((np.zeros((0, 4), np.float32), np.zeros(0, np.float32), np.zeros(0, np.int64)))
            continue
        xywh, mx, lab = p[m, :4], mx[m], lab[m]
        half_w = xywh[:, 2] / np.float32(2)
        half_h = xywh[:, 3] / np.float32(2)
        xyxy = np.stack([xywh[:, 0] - half_w, xywh[:, 1] - half_h, xywh[:, 0] + half_w, xywh[:, 1] + half_h], 1)
        keep = nms(xyxy, mx, iou_thr)
        bx = np.clip(xyxy[keep] / np.float32(img_size), 0.0, 1.0).astype(np.float32)
        outs.append((bx, mx[keep], lab[keep].astype(np.int64)))
    return outs
