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

The helper functions (bbox_iou, bbox2dist, make_anchors, dist2bbox) and the
reference's helper methods (TaskAlignedAssigner.get_pos_mask / get_box_metrics /
select_candidates_in_gts / select_highest_overlaps / get_targets, BboxLoss._df_loss,
v8DetectionLoss.preprocess / bbox_decode) are the reference's tensor utilities with
identical semantics (tests/test_loss_helpers_cpu.py); the HIP path does not call them.  TaskAlignedAssigner and
BboxLoss are callable on their own with the reference's signatures and return
conventions; they run the same HIP kernels on explicit tensors (ym_tal_assign,
ym_bbox_loss_fwd / _bwd).
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from yolomi._lib import YolomiError, call, lib, require_device, stream_ptr


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


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(torch.float32).contiguous()


class TaskAlignedAssigner(nn.Module):
    """Task-aligned assigner (reference :64-270).  As in the reference, `topk` is stored but never
    applied.  `forward` runs the HIP assignment kernels of the fused loss (ym_tal_assign)
    on explicit tensors and returns the reference's 5-tuple; inside v8DetectionLoss the same kernels
    run fused on the head buffer (ym_loss_fwd)."""

    def __init__(self, topk=13, num_classes=80, alpha=1.0, beta=6.0, eps=1e-9):
        super().__init__()
        self.topk, self.num_classes, self.alpha, self.beta, self.eps = topk, num_classes, alpha, beta, eps

    @torch.no_grad()
    def forward(self, pd_scores, pd_bboxes, anc_points, gt_labels, gt_bboxes, mask_gt):
        """-> (target_labels (B,A), target_bboxes (B,A,4), target_scores (B,A,nc), fg_mask (B,A) bool,
        target_gt_idx (B,A) int64), reference :78-180 (including its M = 0 early return :100-108)."""
        require_device(pd_scores, pd_bboxes, anc_points, gt_labels, gt_bboxes, mask_gt)
        self.bs = B = pd_scores.shape[0]
        self.n_max_boxes = M = gt_bboxes.shape[1]
        A, nc = pd_scores.shape[1], pd_scores.shape[2]
        if nc != self.num_classes:
            raise YolomiError(f"pd_scores has {nc} classes, assigner built for {self.num_classes}")
        dev = pd_scores.device
        if M == 0:
            return (torch.full_like(pd_scores[..., 0], self.num_classes).long(), torch.zeros_like(pd_bboxes),
                    torch.zeros_like(pd_scores), torch.zeros_like(pd_scores[..., 0]),
                    torch.zeros_like(pd_scores[..., 0]))
        sc, pb, an = _f32(pd_scores), _f32(pd_bboxes), _f32(anc_points)
        gl, gb = _f32(gt_labels).reshape(B, M), _f32(gt_bboxes).reshape(B, M, 4).clone()   # clone: 16-B aligned
        mg = _f32(mask_gt).reshape(B, M)
        ws_n = lib().ym_tal_assign_workspace_size(B, A, M)
        ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
        t_lab = torch.empty(B, A, dtype=torch.float32, device=dev)
        t_box = torch.empty(B, A, 4, dtype=torch.float32, device=dev)
        t_sc = torch.empty(B, A, nc, dtype=torch.float32, device=dev)
        fg = torch.empty(B, A, dtype=torch.bool, device=dev)
        tgi = torch.empty(B, A, dtype=torch.int64, device=dev)
        call("ym_tal_assign", sc.data_ptr(), pb.data_ptr(), an.data_ptr(), gl.data_ptr(), gb.data_ptr(), mg.data_ptr(),
             B, A, nc, M, float(self.alpha), float(self.beta), float(self.eps), ws.data_ptr(), ws_n, t_lab.data_ptr(), t_box.data_ptr(), t_sc.data_ptr(), fg.data_ptr(),
             tgi.data_ptr(), stream_ptr(dev))
        return t_lab.to(gt_labels.dtype), t_box, t_sc, fg, tgi

    # The reference's step helpers (:182-270), kept for code that calls them directly.  They are tensor
    # utilities on whatever device their inputs live on — the HIP forward above computes the same quantities
    # fused (ym_tal_assign) and does not call them.  get_targets reads self.bs / self.n_max_boxes, which
    # forward sets, as in the reference.
    def get_pos_mask(self, pd_scores, pd_bboxes, gt_labels, gt_bboxes, anc_points, mask_gt):
        """-> (mask_pos (B,A,M) float, align_metric, overlaps), reference :182-194."""
        align_metric, overlaps = self.get_box_metrics(pd_scores, pd_bboxes, gt_labels, gt_bboxes)
        inside = self.select_candidates_in_gts(anc_points, gt_bboxes)
        return inside * mask_gt[:, None, :], align_metric, overlaps

    def get_box_metrics(self, pd_scores, pd_bboxes, gt_labels, gt_bboxes):
        """-> (score^alpha * IoU^beta, IoU clamped at 0), both (B,A,M), reference :196-208."""
        overlaps = bbox_iou(pd_bboxes[:, :, None, :], gt_bboxes[:, None, :, :], xywh=False).squeeze(-1).clamp_(0)
        cls_idx = gt_labels.long()[:, None, :].expand(-1, pd_scores.shape[1], -1)
        return torch.gather(pd_scores, 2, cls_idx).pow(self.alpha) * overlaps.pow(self.beta), overlaps

    def select_candidates_in_gts(self, xy_centers, gt_bboxes, eps=1e-9):
        """(B,A,M) 1.0 where the anchor centre lies strictly inside the box (min side distance > eps),
        in the boxes' dtype, reference :210-224."""
        x, y = xy_centers[None, :, None, 0], xy_centers[None, :, None, 1]
        g = gt_bboxes[:, None, :, :]
        sides = torch.stack((x - g[..., 0], y - g[..., 1], g[..., 2] - x, g[..., 3] - y), -1)
        return (sides.amin(-1) > eps).to(gt_bboxes.dtype)

    def select_highest_overlaps(self, mask_pos, overlaps, n_max_boxes):
        """Anchors claimed by several boxes keep only their highest-IoU box; -> (target_gt_idx, fg_mask,
        mask_pos), reference :226-244."""
        fg_mask = mask_pos.sum(-1)
        if fg_mask.max() > 1:
            shared = (fg_mask[..., None] > 1).expand(-1, -1, n_max_boxes)
            best = torch.zeros_like(mask_pos).scatter_(-1, overlaps.argmax(-1, keepdim=True), 1)
            mask_pos = torch.where(shared, best, mask_pos).float()
            fg_mask = mask_pos.sum(-1)
        return mask_pos.argmax(-1), fg_mask, mask_pos

    def get_targets(self, gt_labels, gt_bboxes, target_gt_idx, fg_mask):
        """-> (labels (B,A), boxes (B,A,4), one-hot scores (B,A,nc) zero off the foreground), reference
        :246-270."""
        rows = target_gt_idx + self.n_max_boxes * torch.arange(self.bs, dtype=torch.int64,
                                                               device=gt_labels.device)[:, None]
        labels = gt_labels.flatten()[rows]
        boxes = gt_bboxes.view(-1, 4)[rows]
        labels.clamp_(0, self.num_classes)
        scores = torch.zeros(*labels.shape, self.num_classes, dtype=torch.float32, device=labels.device)
        scores.scatter_(2, labels[..., None].long(), 1)
        scores = torch.where(fg_mask[..., None].repeat(1, 1, self.num_classes) > 0, scores, 0)
        return labels, boxes, scores.float()


class _BboxLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred_dist, pred_bboxes, anchor_points, target_bboxes, target_scores, tss, fg_mask):
        B, A = fg_mask.shape
        nc = target_scores.shape[-1]
        dev = pred_dist.device
        ins = [_f32(pred_dist).reshape(B, A, 64), _f32(pred_bboxes).reshape(B, A, 4), _f32(anchor_points).reshape(A, 2),
               _f32(target_bboxes).reshape(B, A, 4), _f32(target_scores).reshape(B, A, nc), tss,
               fg_mask.to(torch.uint8).contiguous()]
        ws_n = lib().ym_bbox_loss_workspace_size(B, A)
        ws = torch.empty(max(ws_n, 8), dtype=torch.uint8, device=dev)
        out = torch.empty(2, dtype=torch.float32, device=dev)
        call("ym_bbox_loss_fwd", *[t.data_ptr() for t in ins], B, A, nc, ws.data_ptr(), ws_n, out.data_ptr(),
             stream_ptr(dev))
        ctx.save_for_backward(*ins)
        ctx.meta = (B, A, nc, pred_dist.shape, pred_bboxes.shape)
        return out[0].clone(), out[1].clone()

    @staticmethod
    def backward(ctx, g_iou, g_dfl):
        ins = ctx.saved_tensors
        B, A, nc, sd, sb = ctx.meta
        dev = ins[0].device
        z = torch.zeros((), dtype=torch.float32, device=dev)
        g = torch.stack([(g_iou if g_iou is not None else z).float().reshape(()),
                         (g_dfl if g_dfl is not None else z).float().reshape(())]).contiguous()
        dd = torch.empty(B, A, 64, dtype=torch.float32, device=dev)
        db = torch.empty(B, A, 4, dtype=torch.float32, device=dev)
        call("ym_bbox_loss_bwd", *[t.data_ptr() for t in ins], B, A, nc, g.data_ptr(), dd.data_ptr(), db.data_ptr(),
             stream_ptr(dev))
        return dd.view(sd), db.view(sb), None, None, None, None, None


class BboxLoss(nn.Module):
    """CIoU + DFL box loss (reference :273-324).  `forward` runs ym_bbox_loss_fwd/bwd (the fused
    loss's CIoU and DFL terms on explicit tensors; differentiable in pred_dist and pred_bboxes)."""

    def __init__(self, reg_max=16):
        super().__init__()
        self.reg_max = reg_max

    def forward(self, pred_dist, pred_bboxes, anchor_points, target_bboxes, target_scores, target_scores_sum, fg_mask):
        """-> (loss_iou, loss_dfl), reference :280-310."""
        require_device(pred_dist, pred_bboxes, anchor_points, target_bboxes, target_scores, fg_mask)
        if self.reg_max != 16:
            raise YolomiError("the HIP box loss is specialised for reg_max=16")
        tss = torch.as_tensor(target_scores_sum, dtype=torch.float32, device=pred_dist.device).detach().reshape(1)
        return _BboxLossFn.apply(pred_dist, pred_bboxes, anchor_points, target_bboxes, target_scores,
                                 tss.contiguous(), fg_mask)

    @staticmethod
    def _df_loss(pred_dist, target):
        """Distribution focal loss of (n, reg_max) logits against continuous targets (n, 4) -> (n, 1), reference
        :312-324 (a tensor utility; the HIP box loss computes the same term fused).  Clamps `target` in place, as
        the reference does."""
        target = target.clamp_(0, pred_dist.shape[-1] - 1 - 0.01)
        left = target.long()
        w_left = (left + 1) - target
        ce_l = F.cross_entropy(pred_dist, left.view(-1), reduction="none").view(left.shape)
        ce_r = F.cross_entropy(pred_dist, (left + 1).view(-1), reduction="none").view(left.shape)
        return (ce_l * w_left + ce_r * (1 - w_left)).mean(-1, keepdim=True)


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
        ctx.set_materialize_grads(False)      # items' gradient stays None: no zero-filled (3,) tensor per backward
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

    # The reference's helpers (:501-538), kept for code that calls them directly: tensor utilities on the
    # inputs' device; __call__ does the same work inside ym_loss_fwd and does not call them.
    def preprocess(self, targets_cls, targets_bbox, batch_idx, batch_size, img_size):
        """Padded per-image target table (batch_size, max boxes, 6) = [class, x1, y1, x2, y2 (pixels), 1],
        boxes in each image's original order, rows past an image's count zero; reference :501-527."""
        if len(targets_cls) == 0:
            return torch.zeros(batch_size, 0, 6, device=self.device)
        owner = [batch_idx == i for i in range(batch_size)]
        counts = [int(m.sum()) for m in owner]
        out = torch.zeros(batch_size, max(counts), 6, device=self.device)
        pix = targets_bbox * img_size.repeat(2)[:4]
        for i, (m, n) in enumerate(zip(owner, counts)):
            if n:
                out[i, :n, 0] = targets_cls[m, 0]
                out[i, :n, 1:5] = pix[m]
                out[i, :n, 5] = 1.0
        return out

    def bbox_decode(self, anchor_points, pred_dist, stride_tensor):
        """(B, A, 4*reg_max) side distributions -> xyxy boxes around the anchors (grid units): the softmax
        expectation over the reg_max bins of each side, then dist2bbox; reference :529-538."""
        if self.reg_max > 1:
            b, a, c = pred_dist.shape
            bins = torch.arange(c // 4, device=pred_dist.device, dtype=pred_dist.dtype)
            pred_dist = pred_dist.view(b, a, 4, c // 4).softmax(3).matmul(bins.view(-1, 1)).view(b, a, 4)
        return dist2bbox(pred_dist, anchor_points[None], xywh=False, dim=-1)

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
