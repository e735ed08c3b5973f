"""v8 detection loss — drop-in for the reference's losses/yolo_v8_loss.py.

v8DetectionLoss keeps the reference's constructor, attributes and call
convention (/root/reference/yolo_scratch_cuda/losses/yolo_v8_loss.py:333-538):
`loss, items = criterion(preds, batch)` with `loss = sum(items) * B` and
`items = (7.5*box, 0.5*cls, 1.5*dfl)` detached.  Underneath, the whole loss —
target preprocess, task-aligned assignment with the reference's quirks (no
top-k, sequential forced assignment), CIoU + DFL + BCE and their gradient —
is libyolomi's ym_loss_fwd / ym_loss_bwd on the (B, A, 64+nc) head buffer.
The host synchronises once per call (the largest per-image box count sizes
the GT table) instead of 2*B*M+4 times.

The helper functions (bbox_iou, bbox2dist, make_anchors, dist2bbox) are the
reference's tensor utilities with identical semantics; TaskAlignedAssigner and
BboxLoss carry the reference's hyper-parameters for API compatibility — their
arithmetic lives in the fused kernels.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn as nn

from yolomi._lib import YolomiError, call, lib, stream_ptr


def bbox_iou(box1, box2, xywh=True, GIoU=False, DIoU=False, CIoU=False, eps=1e-7):
    """IoU / GIoU / DIoU / CIoU of broadcastable box sets (reference :12-61)."""
    if xywh:
        (x1, y1, w1, h1), (x2, y2, w2, h2) = box1.chunk(4, -1), box2.chunk(4, -1)
        b1_x1, b1_x2, b1_y1, b1_y2 = x1 - w1 / 2, x1 + w1 / 2, y1 - h1 / 2, y1 + h1 / 2
        b2_x1, b2_x2, b2_y1, b2_y2 = x2 - w2 / 2, x2 + w2 / 2, y2 - h2 / 2, y2 + h2 / 2
    else:
        b1_x1, b1_y1, b1_x2, b1_y2 = box1.chunk(4, -1)
        b2_x1, b2_y1, b2_x2, b2_y2 = box2.chunk(4, -1)
        w1, h1 = b1_x2 - b1_x1, b1_y2 - b1_y1 + eps
        w2, h2 = b2_x2 - b2_x1, b2_y2 - b2_y1 + eps
    inter = (b1_x2.minimum(b2_x2) - b1_x1.maximum(b2_x1)).clamp(0) * \
            (b1_y2.minimum(b2_y2) - b1_y1.maximum(b2_y1)).clamp(0)
    union = w1 * h1 + w2 * h2 - inter + eps
    iou = inter / union
    if CIoU or DIoU or GIoU:
        cw = b1_x2.maximum(b2_x2) - b1_x1.minimum(b2_x1)
        ch = b1_y2.maximum(b2_y2) - b1_y1.minimum(b2_y1)
        if CIoU or DIoU:
            c2 = cw.pow(2) + ch.pow(2) + eps
            rho2 = ((b2_x1 + b2_x2 - b1_x1 - b1_x2).pow(2) + (b2_y1 + b2_y2 - b1_y1 - b1_y2).pow(2)) / 4
            if CIoU:
                v = (4 / math.pi ** 2) * ((w2 / h2).atan() - (w1 / h1).atan()).pow(2)
                with torch.no_grad():
                    alpha = v / (v - iou + (1 + eps))
                return iou - (rho2 / c2 + v * alpha)
            return iou - rho2 / c2
        c_area = cw * ch + eps
        return iou - (c_area - union) / c_area
    return iou


def bbox2dist(anchor_points, bbox, reg_max):
    """xyxy -> clamped ltrb distances (reference :327-330)."""
    x1y1, x2y2 = bbox.chunk(2, -1)
    return torch.cat((anchor_points - x1y1, x2y2 - anchor_points), -1).clamp_(0, reg_max - 0.01)


def make_anchors(feats, strides, grid_cell_offset=0.5):
    """Anchor centres (grid units) and per-anchor strides (reference :541-552)."""
    anchor_points, stride_tensor = [], []
    dtype, device = feats[0].dtype, feats[0].device
    for i, stride in enumerate(strides):
        _, _, h, w = feats[i].shape
        sx = torch.arange(w, device=device, dtype=dtype) + grid_cell_offset
        sy = torch.arange(h, device=device, dtype=dtype) + grid_cell_offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        anchor_points.append(torch.stack((sx, sy), -1).view(-1, 2))
        stride_tensor.append(torch.full((h * w, 1), float(stride), dtype=dtype, device=device))
    return torch.cat(anchor_points), torch.cat(stride_tensor)


def dist2bbox(distance, anchor_points, xywh=True, dim=-1):
    """ltrb distances -> xywh / xyxy (reference :555-564)."""
    lt, rb = distance.chunk(2, dim)
    x1y1 = anchor_points - lt
    x2y2 = anchor_points + rb
    if xywh:
        return torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), dim)
    return torch.cat((x1y1, x2y2), dim)


class TaskAlignedAssigner(nn.Module):
    """Hyper-parameters of the task-aligned assigner (reference :64-76).  As in the reference,
    `topk` is stored but never applied; the assignment runs fused in ym_loss_fwd."""

    def __init__(self, topk=13, num_classes=80, alpha=1.0, beta=6.0, eps=1e-9):
        super().__init__()
        self.topk, self.num_classes, self.alpha, self.beta, self.eps = topk, num_classes, alpha, beta, eps

    def forward(self, *args, **kwargs):
        raise NotImplementedError("the MI355X assigner runs fused inside v8DetectionLoss (ym_loss_fwd)")


class BboxLoss(nn.Module):
    """CIoU + DFL box loss hyper-parameters (reference :273-324); computed in ym_loss_fwd/bwd."""

    def __init__(self, reg_max=16):
        super().__init__()
        self.reg_max = reg_max

    def forward(self, *args, **kwargs):
        raise NotImplementedError("the MI355X box loss runs fused inside v8DetectionLoss (ym_loss_fwd)")


class _LossCtx:
    """Per-shape device workspace of the fused loss."""

    def __init__(self, B, A, M, dev):
        self.B, self.A, self.M = B, A, M
        self.ws_bytes = lib().ym_loss_workspace_size(B, A, M)
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)
        Mm = max(M, 1)
        self.gt_box = torch.empty(B, Mm, 4, dtype=torch.float32, device=dev)
        self.gt_lab = torch.empty(B, Mm, dtype=torch.float32, device=dev)
        self.gt_valid = torch.empty(B, Mm, dtype=torch.int32, device=dev)
        self.out = torch.zeros(8, dtype=torch.float32, device=dev)


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, head, crit, batch, level_hw):
        B, A, no = head.shape
        nc = no - 64
        dev = head.device
        bidx = batch["batch_idx"].to(dev, torch.int64).contiguous()
        cls = batch["cls"].to(dev, torch.int64).reshape(-1).contiguous()
        boxes = batch["bboxes"].to(dev, torch.float32).reshape(-1, 4).contiguous()
        n = int(boxes.shape[0])
        # M = max GTs per image (sizes the assigner): from the batch's host-side "max_gt" when the data
        # path recorded it before the H2D copy (datasets.prepare_batch), else the one host sync
        M = batch.get("max_gt")
        if M is None:
            M = int(torch.bincount(bidx, minlength=B).max().item()) if n else 0
        M = int(M) if n else 0
        key = (B, A, M)
        lc = crit._ctx.get(key)
        if lc is None:
            lc = crit._ctx[key] = _LossCtx(B, A, M, dev)
        nl = len(level_hw)
        lh = (ctypes.c_int * nl)(*[h for h, _ in level_hw])
        lw = (ctypes.c_int * nl)(*[w for _, w in level_hw])
        strides = (ctypes.c_float * nl)(*[float(s) for s in crit.stride[:nl]])
        imgsz_h = float(level_hw[0][0] * float(crit.stride[0]))
        imgsz_w = float(level_hw[0][1] * float(crit.stride[0]))
        st = stream_ptr(dev)
        h = head.detach().contiguous()
        call("ym_loss_fwd", h.data_ptr(), B, A, nc, nl, lh, lw, strides, bidx.data_ptr() if n else None,
             cls.data_ptr() if n else None, boxes.data_ptr() if n else None, n, M, imgsz_h, imgsz_w,
             lc.ws.data_ptr(), lc.ws_bytes, lc.gt_box.data_ptr(), lc.gt_lab.data_ptr(), lc.gt_valid.data_ptr(),
             lc.out.data_ptr(), st)
        ctx.save_for_backward(h)
        ctx.lc, ctx.lv, ctx.strides, ctx.nc = lc, (nl, lh, lw), strides, nc
        crit._last = lc
        loss = lc.out[0].clone()
        items = lc.out[1:4].clone()
        ctx.mark_non_differentiable(items)
        return loss, items

    @staticmethod
    def backward(ctx, gloss, gitems):
        (h,) = ctx.saved_tensors
        lc = ctx.lc
        B, A, no = h.shape
        nl, lh, lw = ctx.lv
        g = gloss.reshape(1).float().contiguous() if gloss is not None else torch.ones(1, device=h.device)
        dhead = torch.empty_like(h)
        call("ym_loss_bwd", h.data_ptr(), B, A, ctx.nc, nl, lh, lw, ctx.strides, lc.M, lc.ws.data_ptr(),
             lc.ws_bytes, lc.gt_box.data_ptr(), lc.gt_lab.data_ptr(), lc.out.data_ptr(), g.data_ptr(),
             dhead.data_ptr(), stream_ptr(h.device))
        return dhead, None, None, None


class v8DetectionLoss:
    """YOLOv8 detection loss (reference :333-538)."""

    def __init__(self, model, tal_topk=10):
        self.bce = nn.BCEWithLogitsLoss(reduction="none")
        self.model = model
        self.tal_topk = tal_topk
        detect = None
        for m in model.modules():
            if type(m).__name__ == "Detect":
                detect = m
                break
        if detect is None:
            raise ValueError("model has no Detect head")
        self.nc = detect.nc
        self.reg_max = detect.reg_max
        self.stride = detect.stride
        self.device = next(model.parameters()).device
        self.assigner = TaskAlignedAssigner(topk=50, num_classes=self.nc, alpha=0.5, beta=4.0)
        self.bbox_loss = BboxLoss(self.reg_max)
        self.epoch = 0
        self.hyp_box = 7.5
        self.hyp_cls = 0.5
        self.hyp_dfl = 1.5
        self._ctx = {}
        self._last = None
        if self.reg_max != 16 or (self.hyp_box, self.hyp_cls, self.hyp_dfl) != (7.5, 0.5, 1.5):
            raise YolomiError("fused loss is specialised for reg_max=16 and gains 7.5/0.5/1.5")

    def _head(self, feats):
        h = getattr(feats[0], "_ym_head", None)
        if h is not None and all(getattr(f, "_ym_head", None) is h for f in feats):
            return h, list(feats[0]._ym_levels)
        # maps that did not come from the yolomi plan: gather them into the (B, A, no) row layout
        B = feats[0].shape[0]
        no = self.nc + 4 * self.reg_max
        head = torch.cat([x.reshape(B, no, -1) for x in feats], 2).permute(0, 2, 1).contiguous()
        return head, [tuple(x.shape[2:]) for x in feats]

    def __call__(self, preds, batch):
        feats = preds[1] if isinstance(preds, tuple) and len(preds) == 2 else preds
        head, level_hw = self._head(feats)
        if not head.is_cuda:
            raise YolomiError("the fused loss runs on the MI355X only (got CPU tensors)")
        loss, items = _LossFn.apply(head, self, batch, level_hw)
        return loss, items

    def assignment(self):
        """(target_gt_idx, fg_mask, target-score magnitude) of the last call, as device tensors (for tests)."""
        lc = self._last
        tgi, fg, nm = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        call("ym_loss_assignment", lc.ws.data_ptr(), lc.B, lc.A, lc.M, ctypes.byref(tgi), ctypes.byref(fg),
             ctypes.byref(nm))
        base = lc.ws.data_ptr()
        n = lc.B * lc.A

        def view(p, dtype):
            off = p.value - base
            return lc.ws[off:off + 4 * n].view(dtype).view(lc.B, lc.A)
        return view(tgi, torch.int32), view(fg, torch.int32), view(nm, torch.float32)
