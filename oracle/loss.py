"""fp32 CPU restatement of v8DetectionLoss — TEST ORACLE ONLY.

Follows /root/reference/yolo_scratch_cuda/losses/yolo_v8_loss.py; line numbers
cited per step.  Quirks reproduced: Q1 no top-k (every
in-box anchor positive), Q2 sequential forced-assignment loops, Q3 GT-axis
normalisation, Q13 loss.sum()*B and gains 7.5/0.5/1.5, Q14 float labels/mask.
Gradients come from CPU autograd through these ops.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .model import anchors as make_anchors

NC, REG_MAX = 5, 16
ALPHA, BETA, EPS = 0.5, 4.0, 1e-9            # TaskAlignedAssigner(topk=50, alpha=.5, beta=4) :363
HYP_BOX, HYP_CLS, HYP_DFL = 7.5, 0.5, 1.5     # :368-370


def bbox_iou(b1, b2, ciou=False, eps=1e-7):
    """xyxy IoU / CIoU with the reference's eps placement (yolo_v8_loss.py:12-61)."""
    b1x1, b1y1, b1x2, b1y2 = b1.chunk(4, -1)
    b2x1, b2y1, b2x2, b2y2 = b2.chunk(4, -1)
    w1, h1 = b1x2 - b1x1, b1y2 - b1y1 + eps
    w2, h2 = b2x2 - b2x1, b2y2 - b2y1 + eps
    inter = (b1x2.minimum(b2x2) - b1x1.maximum(b2x1)).clamp(0) * (b1y2.minimum(b2y2) - b1y1.maximum(b2y1)).clamp(0)
    union = w1 * h1 + w2 * h2 - inter + eps
    iou = inter / union
    if not ciou:
        return iou
    cw = b1x2.maximum(b2x2) - b1x1.minimum(b2x1)
    ch = b1y2.maximum(b2y2) - b1y1.minimum(b2y1)
    c2 = cw.pow(2) + ch.pow(2) + eps
    rho2 = ((b2x1 + b2x2 - b1x1 - b1x2).pow(2) + (b2y1 + b2y2 - b1y1 - b1y2).pow(2)) / 4
    v = (4 / math.pi ** 2) * ((w2 / h2).atan() - (w1 / h1).atan()).pow(2)
    with torch.no_grad():
        alpha = v / (v - iou + (1 + eps))
    return iou - (rho2 / c2 + v * alpha)


def preprocess(cls, boxes, bidx, B, imgsz):
    """(B, M, 6) [cls, x1,y1,x2,y2 (pixels), valid] (yolo_v8_loss.py:501-527)."""
    if len(cls) == 0:
        return torch.zeros(B, 0, 6)
    M = max(int((bidx == i).sum()) for i in range(B))
    out = torch.zeros(B, M, 6)
    scaled = boxes * imgsz.repeat(2)[:4]
    for i in range(B):
        m = bidx == i
        n = int(m.sum())
        if n:
            out[i, :n, 0] = cls[m, 0].float()
            out[i, :n, 1:5] = scaled[m]
            out[i, :n, 5] = 1.0
    return out


def in_gts(xy, gt, eps=1e-9):
    """select_candidates_in_gts (:210-224): strict 'anchor centre inside box'."""
    lt = xy.view(1, -1, 1, 2) - gt[:, None, :, :2]
    rb = gt[:, None, :, 2:] - xy.view(1, -1, 1, 2)
    return torch.cat((lt, rb), -1).amin(-1).gt(eps)


def _highest(mask_pos, overlaps):
    """select_highest_overlaps (:226-244)."""
    fg = mask_pos.sum(-1)
    if fg.numel() and fg.max() > 1:
        multi = (fg.unsqueeze(-1) > 1).expand_as(mask_pos)
        best = torch.zeros_like(mask_pos).scatter_(-1, overlaps.argmax(-1, keepdim=True), 1)
        mask_pos = torch.where(multi, best, mask_pos).float()
        fg = mask_pos.sum(-1)
    return mask_pos.argmax(-1), fg, mask_pos


@torch.no_grad()
def assign(pd_scores, pd_bboxes, anc, gt_labels, gt_bboxes, mask_gt):
    """TaskAlignedAssigner.forward (:78-180). Returns labels, bboxes, scores, fg(bool), tgi."""
    B, A, nc = pd_scores.shape
    M = gt_bboxes.shape[1]
    if M == 0:
        return (torch.full((B, A), nc, dtype=torch.long), torch.zeros(B, A, 4), torch.zeros(B, A, nc),
                torch.zeros(B, A), torch.zeros(B, A))
    overlaps = bbox_iou(pd_bboxes.unsqueeze(2), gt_bboxes.unsqueeze(1)).squeeze(-1).clamp(0)      # :199
    cls_s = pd_scores.gather(-1, gt_labels.unsqueeze(1).expand(-1, A, -1).long())                   # :202-203
    align = cls_s.pow(ALPHA) * overlaps.pow(BETA)                                                   # :206
    inbox = in_gts(anc, gt_bboxes)
    mask_pos = inbox * mask_gt.unsqueeze(1)                                                         # :192
    # loop 1 (:117-139): independent per gt column
    for b in range(B):
        for g in range(M):
            if mask_gt[b, g] and mask_pos[b, :, g].sum() == 0:
                ib = inbox[b, :, g]
                a = (overlaps[b, :, g] * ib.float()).argmax() if ib.sum() > 0 else overlaps[b, :, g].argmax()
                mask_pos[b, a, g] = 1.0
    tgi, fg, mask_pos = _highest(mask_pos, overlaps)
    # loop 2 (:146-162): sequential; tgi/fg edits feed later checks, only mask_pos survives
    for b in range(B):
        for g in range(M):
            if mask_gt[b, g]:
                if not (tgi[b][fg[b] > 0] == g).any():
                    a = overlaps[b, :, g].argmax()
                    mask_pos[b, a, g] = 1.0
                    tgi[b, a] = g
                    fg[b, a] = 1
    tgi, fg, mask_pos = _highest(mask_pos, overlaps)                                                # :165
    flat = tgi + torch.arange(B)[:, None] * M                                                       # get_targets :246-270
    t_labels = gt_labels.flatten()[flat].clamp(0, nc)
    t_bboxes = gt_bboxes.view(-1, 4)[flat]
    ts = torch.zeros(B, A, nc).scatter_(2, t_labels.unsqueeze(-1).long(), 1)
    ts = torch.where(fg[:, :, None].repeat(1, 1, nc) > 0, ts, 0)
    align = align * mask_pos                                                                        # :173-178
    pam = align.amax(-1, keepdim=True)
    pov = (overlaps * mask_pos).amax(-1, keepdim=True)
    norm = (align * pov / (pam + EPS)).amax(-1).unsqueeze(-1)
    return t_labels, t_bboxes, ts * norm, fg.bool(), tgi


def df_loss(pd, t):
    """_df_loss (:312-324)."""
    t = t.clamp(0, pd.shape[-1] - 1 - 0.01)
    tl = t.long()
    tr = tl + 1
    wl = tr - t
    wr = 1 - wl
    ll = F.cross_entropy(pd, tl.view(-1), reduction="none").view(tl.shape) * wl
    lr = F.cross_entropy(pd, tr.view(-1), reduction="none").view(tl.shape) * wr
    return (ll + lr).mean(-1, keepdim=True)


def v8_loss(feats, batch, strides=(8.0, 16.0, 32.0), nc=NC, return_internals=False):
    """v8DetectionLoss.__call__ (:372-499) on the list of 3 head maps (B, 64+nc, H, W)."""
    B = feats[0].shape[0]
    no = nc + 4 * REG_MAX
    pd_distri, pd_scores = torch.cat([x.view(B, no, -1) for x in feats], 2).split((4 * REG_MAX, nc), 1)
    pd_scores = pd_scores.permute(0, 2, 1).contiguous()
    pd_distri = pd_distri.permute(0, 2, 1).contiguous()
    imgsz = torch.tensor(feats[0].shape[2:], dtype=torch.float32) * strides[0]
    tg = preprocess(batch["cls"], batch["bboxes"], batch["batch_idx"], B, imgsz)
    gt_labels, gt_bboxes, mask_gt = tg.split((1, 4, 1), 2)
    mask_gt = mask_gt.gt(0).float().squeeze(-1)
    anc, st = make_anchors([x.shape[2:] for x in feats], strides)
    A = anc.shape[0]
    proj = torch.arange(REG_MAX, dtype=torch.float32)
    d = pd_distri.view(B, A, 4, REG_MAX).softmax(3).matmul(proj.view(-1, 1)).view(B, A, 4)       # :529-538
    lt, rb = d.chunk(2, -1)
    pred_bboxes = torch.cat((anc - lt, anc + rb), -1)
    t_labels, t_bboxes, t_scores, fg, tgi = assign(
        pd_scores.detach().sigmoid(), (pred_bboxes * st).detach(), anc * st, gt_labels.squeeze(-1), gt_bboxes, mask_gt)
    tss = max(t_scores.sum(), 1)                                                                   # :472
    l_cls = F.binary_cross_entropy_with_logits(pd_scores, t_scores, reduction="none").sum() / tss
    zero = pd_scores.sum() * 0
    l_box, l_dfl = zero, zero
    if fg.sum():
        t_b = t_bboxes / st
        w = t_scores.sum(-1)[fg].unsqueeze(-1)
        iou = bbox_iou(pred_bboxes[fg], t_b[fg], ciou=True)
        l_box = ((1.0 - iou) * w).sum() / tss
        x1y1, x2y2 = t_b.chunk(2, -1)
        t_ltrb = torch.cat((anc - x1y1, x2y2 - anc), -1).clamp(0, REG_MAX - 1 - 0.01)             # bbox2dist :327-330
        l_dfl = (df_loss(pd_distri[fg].view(-1, REG_MAX), t_ltrb[fg]) * w).sum() / tss
    items = torch.stack((l_box * HYP_BOX, l_cls * HYP_CLS, l_dfl * HYP_DFL))
    loss = items.sum() * B
    if return_internals:
        return loss, items.detach(), dict(fg=fg, tgi=tgi, target_scores=t_scores, tss=tss)
    return loss, items.detach()
