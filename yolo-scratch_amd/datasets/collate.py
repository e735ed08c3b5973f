"""Batch-dict contract of the reference loader.

collate_fn_cuda follows crater_dataset_cuda.py:289-346: stack images, emit
(batch_idx, cls, bboxes) with boxes converted from normalised cxcywh to xyxy
and clamped to [0, 1] (:313-322).  The crater CSV/image dataset itself
(CraterDatasetCUDA, :26-286) is a "next" row; here it fails
loudly instead of silently producing something else.
"""
from __future__ import annotations

import torch


def collate_fn_cuda(batch):
    imgs, boxes_list, labels_list, _ = zip(*batch)
    imgs = torch.stack(imgs, 0)
    bidx, cls, bboxes = [], [], []
    for i, (boxes, labels) in enumerate(zip(boxes_list, labels_list)):
        if len(boxes) == 0:
            continue
        bidx.append(torch.full((len(boxes),), i, dtype=torch.long))
        cls.append(labels.reshape(-1, 1).long())
        c, wh = boxes[:, :2], boxes[:, 2:4]
        bboxes.append(torch.cat((c - wh / 2, c + wh / 2), 1).clamp(0.0, 1.0))
    if not bidx:
        return {"img": imgs, "batch_idx": torch.zeros((0,), dtype=torch.long),
                "cls": torch.zeros((0, 1), dtype=torch.long), "bboxes": torch.zeros((0, 4), dtype=torch.float32)}
    return {"img": imgs, "batch_idx": torch.cat(bidx), "cls": torch.cat(cls), "bboxes": torch.cat(bboxes).float()}


class CraterDatasetCUDA(torch.utils.data.Dataset):
    def __init__(self, *a, **k):
        raise NotImplementedError("crater CSV/image loader is not part of this build yet; use --synthetic N")
