"""Batch-dict contract of the reference loader.

collate_fn_cuda follows crater_dataset_cuda.py:289-346: stack images, emit
(batch_idx, cls, bboxes) with boxes converted from normalised cxcywh to xyxy
and clamped to [0, 1] (:313-322).  The crater CSV/image dataset itself
(CraterDatasetCUDA, :26-286) lives in datasets/crater.py.
"""
from __future__ import annotations

import torch


def collate_fn_cuda(batch, img_size=None):
    """Batch dict of the reference collate (:289-346).  Images that are raw uint8 (1, h0, w0)
    (datasets.crater.CraterDatasetCUDA) are packed for the GPU resize instead of stacked:
    the dict then carries img_u8 / img_meta / img_size until datasets.prepare_batch moves it to
    the device and produces img (B, 1, S, S) fp32."""
    imgs, boxes_list, labels_list, _ = zip(*batch)
    if imgs and imgs[0].dtype == torch.uint8:
        from .crater import pack_images
        size = img_size or getattr(imgs[0], "img_size", None)
        if size is None:
            raise ValueError("collate_fn_cuda: raw uint8 images need img_size (functools.partial(collate_fn_cuda, "
                             "img_size=S))")
        out = pack_images(imgs, size)
    else:
        out = {"img": torch.stack(imgs, 0)}
    bidx, cls, bboxes = [], [], []
    for i, (boxes, labels) in enumerate(zip(boxes_list, labels_list)):
        if len(boxes) == 0:
            continue
        bidx.append(torch.full((len(boxes),), i, dtype=torch.long))
        cls.append(labels.reshape(-1, 1).long())
        c, wh = boxes[:, :2], boxes[:, 2:4]
        bboxes.append(torch.cat((c - wh / 2, c + wh / 2), 1).clamp(0.0, 1.0))
    if not bidx:
        out.update({"batch_idx": torch.zeros((0,), dtype=torch.long), "cls": torch.zeros((0, 1), dtype=torch.long),
                    "bboxes": torch.zeros((0, 4), dtype=torch.float32)})
        return out
    out.update({"batch_idx": torch.cat(bidx), "cls": torch.cat(cls), "bboxes": torch.cat(bboxes).float()})
    return out
