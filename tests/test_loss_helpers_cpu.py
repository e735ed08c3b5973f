"""The reference's loss helper methods kept on the drop-in classes (TaskAlignedAssigner.get_pos_mask /
get_box_metrics / select_candidates_in_gts / select_highest_overlaps / get_targets, BboxLoss._df_loss,
v8DetectionLoss.preprocess / bbox_decode: reference losses/yolo_v8_loss.py:182-270, 312-324, 501-538).

They are tensor utilities (the HIP path computes the same quantities fused), so they are checked on the CPU
against the oracle restatement (oracle/loss.py, pinned to the reference by tests/test_oracle.py): each helper
on its own, and the reference's whole assignment composed from them against oracle.assign.
"""
import pytest
import torch

from oracle import loss as OL


def _assigner():
    from losses.yolo_v8_loss import TaskAlignedAssigner
    return TaskAlignedAssigner(topk=50, num_classes=OL.NC, alpha=OL.ALPHA, beta=OL.BETA, eps=OL.EPS)


def _case(seed, B=3, A=400, M=5, side=20):
    g = torch.Generator().manual_seed(seed)
    ys, xs = torch.meshgrid(torch.arange(side) + 0.5, torch.arange(side) + 0.5, indexing="ij")
    anc = torch.stack((xs, ys), -1).view(-1, 2)[:A]
    scores = torch.rand(B, A, OL.NC, generator=g)
    c = torch.rand(B, A, 2, generator=g) * side
    wh = torch.rand(B, A, 2, generator=g) * 6 + 0.5
    pd_boxes = torch.cat((c - wh / 2, c + wh / 2), -1)
    gc = torch.rand(B, M, 2, generator=g) * side
    gwh = torch.rand(B, M, 2, generator=g) * 8 + 1.0
    gt_boxes = torch.cat((gc - gwh / 2, gc + gwh / 2), -1)
    gt_labels = torch.randint(0, OL.NC, (B, M), generator=g).float()
    mask_gt = (torch.rand(B, M, generator=g) > 0.25).float()
    return scores, pd_boxes, anc, gt_labels, gt_boxes, mask_gt


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_candidates_and_highest_overlaps_vs_oracle(seed):
    s, pb, anc, gl, gb, mg = _case(seed)
    ta = _assigner()
    inside = ta.select_candidates_in_gts(anc, gb)
    assert inside.dtype == gb.dtype
    assert torch.equal(inside.bool(), OL.in_gts(anc, gb))
    align, ov = ta.get_box_metrics(s, pb, gl, gb)
    ref_ov = OL.bbox_iou(pb.unsqueeze(2), gb.unsqueeze(1)).squeeze(-1).clamp(0)
    assert torch.equal(ov, ref_ov)
    ref_align = s.gather(-1, gl.unsqueeze(1).expand(-1, s.shape[1], -1).long()).pow(OL.ALPHA) * ref_ov.pow(OL.BETA)
    assert torch.equal(align, ref_align)
    mask_pos, align2, ov2 = ta.get_pos_mask(s, pb, gl, gb, anc, mg)
    assert torch.equal(mask_pos, OL.in_gts(anc, gb) * mg.unsqueeze(1)) and torch.equal(align2, align)
    # several anchors inside several boxes: the highest-IoU box wins
    tgi, fg, mp = ta.select_highest_overlaps(mask_pos, ov, gb.shape[1])
    rtgi, rfg, rmp = OL._highest(mask_pos, ov)
    assert torch.equal(tgi, rtgi) and torch.equal(fg, rfg) and torch.equal(mp, rmp)


@pytest.mark.parametrize("seed", [3, 4, 5])
def test_assignment_composed_from_helpers_vs_oracle(seed):
    """The reference forward (:78-180) written with the helpers == oracle.assign (bit-exact)."""
    s, pb, anc, gl, gb, mg = _case(seed)
    ta = _assigner()
    ta.bs, ta.n_max_boxes = s.shape[0], gb.shape[1]
    B, M = ta.bs, ta.n_max_boxes
    mask_pos, align, ov = ta.get_pos_mask(s, pb, gl, gb, anc, mg)
    for b in range(B):
        for g in range(M):
            if mg[b, g] and mask_pos[b, :, g].sum() == 0:
                inside = ta.select_candidates_in_gts(anc, gb[b:b + 1, g:g + 1]).squeeze(0).squeeze(-1)
                best = (ov[b, :, g] * inside).argmax() if inside.sum() > 0 else ov[b, :, g].argmax()
                mask_pos[b, best, g] = 1.0
    tgi, fg, mask_pos = ta.select_highest_overlaps(mask_pos, ov, M)
    for b in range(B):
        for g in range(M):
            if mg[b, g] and not (tgi[b][fg[b] > 0] == g).any():
                best = ov[b, :, g].argmax()
                mask_pos[b, best, g] = 1.0
                tgi[b, best] = g
                fg[b, best] = 1
    tgi, fg, mask_pos = ta.select_highest_overlaps(mask_pos, ov, M)
    labels, boxes, scores = ta.get_targets(gl, gb, tgi, fg)
    align = align * mask_pos
    norm = (align * (ov * mask_pos).amax(-1, keepdim=True) / (align.amax(-1, keepdim=True) + ta.eps)).amax(-1)
    scores = scores * norm.unsqueeze(-1)
    r = OL.assign(s, pb, anc, gl, gb, mg)
    assert torch.equal(labels, r[0]) and torch.equal(boxes, r[1]) and torch.equal(scores, r[2])
    assert torch.equal(fg.bool(), r[3]) and torch.equal(tgi, r[4])


def test_df_loss_vs_oracle():
    from losses.yolo_v8_loss import BboxLoss
    g = torch.Generator().manual_seed(7)
    pd = torch.randn(200, 16, generator=g)
    t = torch.rand(50, 4, generator=g) * 17 - 0.5          # some targets outside [0, 15): clamped
    got = BboxLoss._df_loss(pd, t.clone())
    assert got.shape == (50, 1)
    assert torch.equal(got, OL.df_loss(pd, t.clone()))


def _crit():
    import yaml
    from pathlib import Path
    from models import build_yolo11
    from losses import v8DetectionLoss
    cfg = yaml.safe_load((Path(__file__).resolve().parents[1] / "yolo-scratch_amd" / "configs" /
                          "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "n"
    return v8DetectionLoss(build_yolo11(cfg, ch=1, nc=OL.NC))


def test_preprocess_and_bbox_decode():
    crit = _crit()
    g = torch.Generator().manual_seed(11)
    n = 17
    cls = torch.randint(0, OL.NC, (n, 1), generator=g).float()
    xy = torch.rand(n, 2, generator=g) * 0.7
    boxes = torch.cat((xy, xy + torch.rand(n, 2, generator=g) * 0.3), -1)
    bidx = torch.tensor([0, 2, 2, 0, 3, 2, 0, 0, 3, 2, 2, 0, 3, 3, 0, 2, 2])
    img = torch.tensor([320.0, 320.0])
    got = crit.preprocess(cls, boxes, bidx, 4, img)
    assert torch.equal(got, OL.preprocess(cls, boxes, bidx, 4, img))
    assert got[1].abs().sum() == 0                                      # image 1 has no boxes
    assert crit.preprocess(cls[:0], boxes[:0], bidx[:0], 4, img).shape == (4, 0, 6)
    # bbox_decode: the softmax expectation of each side's 16 bins, then xyxy around the anchor
    pd = torch.randn(2, 30, 64, generator=g)
    anc = torch.rand(30, 2, generator=g) * 40
    got = crit.bbox_decode(anc, pd, None)
    p = pd.view(2, 30, 4, 16).softmax(-1)
    d = (p * torch.arange(16.0)).sum(-1)
    ref = torch.cat((anc - d[..., :2], anc + d[..., 2:]), -1)
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-5)
