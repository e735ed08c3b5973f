"""CPU restatement of the reference data path (TEST INFRASTRUCTURE ONLY — imported by tests/).

Follows /root/reference/yolo_scratch_cuda/datasets/crater_dataset_cuda.py:
  annotations  _load_annotations :77-124 (glob altitude*/longitude*/truth/detections.csv, group by
               inputImage, class = crater_classification or 2 (B) when missing / -1, w/h = 2 x the
               ellipse semi-axes)
  image        load_image :162-186 (cv2.imdecode IMREAD_GRAYSCALE, stretch to S x S with
               cv2.resize INTER_LINEAR unless already S x S), __getitem__ :253 (/255 -> fp32)
  targets      __getitem__ :262-279 (normalise by the ORIGINAL size; cx, cy clamped to [0, 1],
               w, h to [0.01, 1])
The arithmetic lives in OpenCV (requirements.txt:3 `opencv-python`, unpinned), which is not
installed here: `resize_linear_u8` restates OpenCV's fixed-point INTER_LINEAR for 8-bit images
(resize.cpp resizeGeneric_: 11-bit coefficients rounded half-to-even, exact horizontal pass, the
SIMD vertical rounding ((b0*(h0>>4))>>16 + (b1*(h1>>4))>>16 + 2) >> 2) and `gray_from_rgb`
OpenCV's RGB->GRAY fixed point (R*4899 + G*9617 + B*1868 + 8192) >> 14.  PARITY UNPINNED against
cv2 itself (no cv2 build and no reference fixture for this path); the GPU kernel is checked
bit-exact against this restatement.
"""
from __future__ import annotations

import glob
from pathlib import Path

import numpy as np


def _coeffs(n_out: int, n_in: int):
    scale = n_in / n_out                                   # double, as OpenCV's scale_x
    d = np.arange(n_out, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0.0, 0
    hi = s >= n_in - 1
    f[hi], s[hi] = 0.0, n_in - 1
    a0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    return s, np.minimum(s + 1, n_in - 1), a0, a1


def resize_linear_u8(im: np.ndarray, size: int) -> np.ndarray:
    """uint8 (h0, w0) -> uint8 (size, size), OpenCV INTER_LINEAR fixed point (see module doc)."""
    h0, w0 = im.shape
    if h0 == size and w0 == size:
        return im.copy()
    sx, sx1, a0, a1 = _coeffs(size, w0)
    sy, sy1, b0, b1 = _coeffs(size, h0)
    src = im.astype(np.int64)
    h = src[:, sx] * a0 + src[:, sx1] * a1                 # (h0, size) horizontal pass
    top = (b0[:, None] * (h[sy] >> 4)) >> 16
    bot = (b1[:, None] * (h[sy1] >> 4)) >> 16
    return np.clip((top + bot + 2) >> 2, 0, 255).astype(np.uint8)


def gray_from_rgb(rgb: np.ndarray) -> np.ndarray:
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((r * 4899 + g * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)


def image_tensor(im_u8: np.ndarray, size: int) -> np.ndarray:
    """(1, size, size) fp32 in [0, 1] (load_image + __getitem__ :253-254)."""
    return (resize_linear_u8(im_u8, size).astype(np.float32) / np.float32(255.0))[None]


def load_annotations(data_dir):
    """[(image path, [(cx, cy, w, h, class)])] in the reference's order (:77-124)."""
    import pandas as pd
    out = []
    for csv_path in glob.glob(str(Path(data_dir) / "altitude*/longitude*/truth/detections.csv")):
        csv_path = Path(csv_path)
        parent = csv_path.parent.parent
        df = pd.read_csv(csv_path)
        for img_name, g in df.groupby("inputImage"):
            p = parent / img_name
            if not p.exists():
                continue
            anns = []
            for _, row in g.iterrows():
                c = row.get("crater_classification", -1)
                c = 2 if (pd.isna(c) or c == -1) else int(c)
                anns.append((float(row["ellipseCenterX(px)"]), float(row["ellipseCenterY(px)"]),
                             2.0 * float(row["ellipseSemimajor(px)"]), 2.0 * float(row["ellipseSemiminor(px)"]), c))
            if anns:
                out.append((str(p), anns))
    return out


def targets(anns, h0: int, w0: int):
    """boxes (n, 4) normalised cxcywh (clamped as :271-274) and labels (n,) int64."""
    b = []
    for cx, cy, w, h, _ in anns:
        b.append([max(0.0, min(1.0, cx / w0)), max(0.0, min(1.0, cy / h0)),
                  max(0.01, min(1.0, w / w0)), max(0.01, min(1.0, h / h0))])
    return np.asarray(b, np.float32).reshape(-1, 4), np.asarray([a[4] for a in anns], np.int64)
