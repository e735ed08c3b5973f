"""Synthetic batches with the exact contract of the reference collate function.

The reference batch dict is produced by ``collate_fn_cuda``
(/root/reference/yolo_scratch_cuda/datasets/crater_dataset_cuda.py:289-346):

    img       (B, 1, S, S) float32 in [0, 1)
    batch_idx (N,)  int64   image index of each box
    cls       (N, 1) int64  class id
    bboxes    (N, 4) float32 normalised xyxy, clamped to [0, 1] (:319-322)

There is no dataset in this environment, so training and benchmarking use the
synthetic distribution of SURVEY.md §8(d): 1..max_gt boxes per image, centres
U(0,1)^2, w/h log-uniform in [0.02, 0.5], class U{0..nc-1}.  Everything is
drawn from a CPU ``torch.Generator`` so a seed reproduces a batch bit-exactly
on any host.
"""
from __future__ import annotations

import math

import torch


def synth_targets(batch: int, seed: int, max_gt: int = 20, nc: int = 5):
    g = torch.Generator().manual_seed(seed)
    counts = torch.randint(1, max_gt + 1, (batch,), generator=g)
    idx, cls, boxes = [], [], []
    lo, hi = math.log(0.02), math.log(0.5)
    for i in range(batch):
        n = int(counts[i])
        c = torch.rand(n, 2, generator=g)
        wh = torch.exp(lo + (hi - lo) * torch.rand(n, 2, generator=g))
        xyxy = torch.cat((c - wh / 2, c + wh / 2), 1).clamp_(0.0, 1.0)
        idx.append(torch.full((n,), i, dtype=torch.long))
        cls.append(torch.randint(0, nc, (n, 1), generator=g))
        boxes.append(xyxy)
    return torch.cat(idx), torch.cat(cls), torch.cat(boxes).float()


def synth_batch(batch: int, imgsz: int, seed: int, max_gt: int = 20, nc: int = 5, ch: int = 1):
    """One collate-compatible batch dict (CPU tensors)."""
    g = torch.Generator().manual_seed(seed ^ 0x5EED)
    img = torch.rand(batch, ch, imgsz, imgsz, generator=g)
    bidx, cls, boxes = synth_targets(batch, seed, max_gt, nc)
    return {"img": img, "batch_idx": bidx, "cls": cls, "bboxes": boxes}


def synth_eval_preds(batch: int, anchors: int, nc: int = 5, img_size: int = 640,
                     objects: int = 10, seed: int = 0) -> torch.Tensor:
    """Anchor-major decoded predictions (B, A, 4+nc): xywh pixels + sigmoid scores.

    Boxes are clustered around ``objects`` per image so NMS has real work to do;
    per-class scores are sigmoid(1.5*randn - 2) (≈80 % of anchors above 0.25).
    Max scores are made pairwise distinct per image so the reference's unstable
    argsort (train_yolo11_cuda.py:377) has a unique answer.
    """
    g = torch.Generator().manual_seed(seed)
    out = torch.empty(batch, anchors, 4 + nc)
    for b in range(batch):
        ctr = torch.rand(objects, 2, generator=g) * img_size
        size = 16 + torch.rand(objects, 2, generator=g) * (img_size / 4)
        owner = torch.randint(0, objects, (anchors,), generator=g)
        jit = torch.randn(anchors, 4, generator=g)
        xy = ctr[owner] + jit[:, :2] * size[owner] * 0.15
        wh = size[owner] * (1.0 + 0.2 * jit[:, 2:])
        scores = torch.sigmoid(1.5 * torch.randn(anchors, nc, generator=g) - 2.0)
        # make the per-anchor max unique: rank-based distinct values keep the order
        mx, arg = scores.max(1)
        order = torch.argsort(mx, stable=True)
        ranks = torch.empty_like(order)
        ranks[order] = torch.arange(anchors)
        distinct = 0.001 + 0.998 * (ranks.float() + 1) / (anchors + 1)
        scores = scores * (0.999 * distinct / mx).unsqueeze(1)   # others strictly below the max
        scores[torch.arange(anchors), arg] = distinct
        out[b, :, :2] = xy
        out[b, :, 2:4] = wh.abs()
        out[b, :, 4:] = scores
    return out
