"""The drop-in boundary's standalone callables against the reference (fixtures made by running it):

* TaskAlignedAssigner.forward (losses/yolo_v8_loss.py:78-180) on the assigner's own captured inputs
  -> the reference's 5-tuple: fg_mask, target_gt_idx and target_labels / target_bboxes bit-exact,
  target_scores within 1e-5; and its M = 0 early return;
* BboxLoss.forward (:280-324): (loss_iou, loss_dfl) within 1e-5 and their gradient w.r.t. pred_dist
  and pred_bboxes within 1e-4;
* Detect called on its own (models/yolo11_modules.py:237-266): train maps, input / parameter
  gradients, BN running stats, the eval (y, maps) — 16-bit conv path, 1e-2 / 2e-2;
* Concat (:277-285): exact.
"""
import numpy as np
import pytest
import torch

from test_gpu_model import rel

pytestmark = pytest.mark.gpu


def test_task_aligned_assigner_forward_vs_reference(golden):
    from losses import TaskAlignedAssigner
    d = golden("assigner.npz")
    ins = [torch.from_numpy(d["as_" + k]).cuda() for k in
           ("pd_scores", "pd_bboxes", "anc_points", "gt_labels", "gt_bboxes", "mask_gt")]
    tal = TaskAlignedAssigner(topk=50, num_classes=5, alpha=0.5, beta=4.0)
    tl, tb, ts, fg, tgi = tal(*ins)
    assert fg.dtype == torch.bool and tgi.dtype == torch.int64 and tl.dtype == ins[3].dtype
    np.testing.assert_array_equal(fg.cpu().numpy(), d["fg"])
    np.testing.assert_array_equal(tgi.cpu().numpy(), d["tgi"])
    np.testing.assert_array_equal(tl.cpu().numpy(), d["target_labels"])
    np.testing.assert_array_equal(tb.cpu().numpy(), d["target_bboxes"])
    torch.testing.assert_close(ts.cpu(), torch.from_numpy(d["target_scores"]), rtol=1e-5, atol=1e-6)
    # M = 0: the reference's early return (:100-108) — labels = nc (long), everything else zero
    empty = tal(ins[0], ins[1], ins[2], ins[3][:, :0], ins[4][:, :0], ins[5][:, :0])
    assert empty[0].dtype == torch.int64 and bool((empty[0] == 5).all())
    assert all(float(t.abs().sum()) == 0 for t in empty[1:])


def test_bbox_loss_forward_backward_vs_reference(golden):
    from losses import BboxLoss
    d = golden("assigner.npz")
    pd = torch.from_numpy(d["bl_pred_dist"]).cuda().requires_grad_(True)
    pb = torch.from_numpy(d["bl_pred_bboxes"]).cuda().requires_grad_(True)
    rest = [torch.from_numpy(d[k]).cuda() for k in ("bl_anchor_points", "bl_target_bboxes", "bl_target_scores")]
    tss = torch.tensor(float(d["bl_tss"]), device="cuda")
    fg = torch.from_numpy(d["bl_fg_mask"]).cuda()
    li, ld = BboxLoss(16)(pd, pb, rest[0], rest[1], rest[2], tss, fg)
    torch.testing.assert_close(li.cpu(), torch.from_numpy(d["bl_loss_iou"]), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(ld.cpu(), torch.from_numpy(d["bl_loss_dfl"]), rtol=1e-5, atol=1e-7)
    (1.3 * li + 0.7 * ld).backward()
    torch.testing.assert_close(pd.grad.cpu(), torch.from_numpy(d["bl_dpred_dist"]), rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(pb.grad.cpu(), torch.from_numpy(d["bl_dpred_bboxes"]), rtol=1e-4, atol=1e-8)
    # target_scores_sum given as a Python number (the reference's max(tensor, 1) may return int 1)
    li2, ld2 = BboxLoss(16)(pd.detach(), pb.detach(), rest[0], rest[1], rest[2], float(d["bl_tss"]), fg)
    assert torch.equal(li2, li.detach()) and torch.equal(ld2, ld.detach())


def _detect(d):
    from models import Detect
    det = Detect(5, (32, 64, 128))
    det.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("p:")})
    det.stride = torch.tensor([8.0, 16.0, 32.0])
    for m in det.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.eps, m.momentum = 1e-3, 0.03
    return det.cuda()


def test_detect_standalone_train_eval_vs_reference(golden):
    d = golden("detect.npz")
    det = _detect(d).train()
    xs = [torch.from_numpy(d[f"x{i}"]).cuda().requires_grad_(True) for i in range(3)]
    ys = det(xs)
    assert isinstance(ys, list) and len(ys) == 3
    for i in range(3):
        assert ys[i].shape == tuple(d[f"y{i}"].shape)
        assert rel(ys[i], d[f"y{i}"]) < 1e-2, (i, rel(ys[i], d[f"y{i}"]))
    torch.autograd.backward(ys, [torch.from_numpy(d[f"dy{i}"]).cuda() for i in range(3)])
    for i in range(3):
        assert rel(xs[i].grad, d[f"dx{i}"]) < 2e-2, (i, rel(xs[i].grad, d[f"dx{i}"]))
    scale = max(float(np.linalg.norm(d[k])) for k in d.files if k.startswith("g:"))
    for k, p in det.named_parameters():
        if not p.requires_grad:
            continue
        ref = d["g:" + k]
        err = float((p.grad.double().cpu() - torch.from_numpy(ref).double()).norm())
        assert err < 3e-2 * max(float(np.linalg.norm(ref)), 5e-3 * scale), (k, err)
    sd = det.state_dict()
    for k in [n for n in d.files if n.startswith("s:")]:
        assert rel(sd[k[2:]], d[k]) < 1e-2, k
    det.eval()
    with torch.no_grad():
        y, maps = det([x.detach() for x in xs])
    assert rel(y, d["eval_y"]) < 1e-2, rel(y, d["eval_y"])
    for i in range(3):
        assert rel(maps[i], d[f"eval_map{i}"]) < 1e-2
    # Detect.inference on its own maps equals the eval forward's y
    torch.testing.assert_close(det.inference([m.clone() for m in maps]), y, rtol=1e-6, atol=1e-5)


def test_concat_standalone_exact(golden):
    from models import Concat
    d = golden("detect.npz")
    a = torch.from_numpy(d["cat_a"]).cuda().requires_grad_(True)
    b = torch.from_numpy(d["cat_b"]).cuda().requires_grad_(True)
    out = Concat(1)([a, b])
    np.testing.assert_array_equal(out.detach().cpu().numpy(), d["cat_out1"])
    out2 = Concat(2)([a, a[:, :, :2]])
    np.testing.assert_array_equal(out2.detach().cpu().numpy(), d["cat_out2"])
    g = torch.randn(out.shape, device="cuda")
    out.backward(g)
    torch.testing.assert_close(a.grad, g[:, :3], rtol=0, atol=0)
    torch.testing.assert_close(b.grad, g[:, 3:], rtol=0, atol=0)
