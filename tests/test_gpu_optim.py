"""FusedAdamW (yolomi/optim.py, csrc/optim.hip) against torch's own clip_grad_norm_ + AdamW.

The reference's optimizer tail is `clip_grad_norm_(params, 10.0)` + `optim.AdamW(lr, weight_decay)`
(train_yolo11_cuda.py:58-62, 440-451); the fused form must take the same steps.  fp32 throughout:
tolerance 1e-5 relative (the kernel's update and the norm's summation order round differently from
ATen's single-tensor loop), and the state_dict must be interchangeable with torch.optim.AdamW's.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(64, 32, 3, 3), (5,), (64,), (7, 3), (128, 96, 1, 1), (1,)]


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(s, generator=g).cuda().requires_grad_(True) for s in SHAPES]


def _grads(step, scale):
    g = torch.Generator().manual_seed(100 + step)
    return [torch.randn(s, generator=g).cuda() * scale for s in SHAPES]


@pytest.mark.parametrize("clip,scale", [(None, 1.0), (10.0, 1.0), (10.0, 0.01), (0.5, 3.0)])
def test_fused_adamw_matches_torch(clip, scale):
    from yolomi.optim import FusedAdamW
    a, b = _params(0), _params(0)
    ref = torch.optim.AdamW(a, lr=1e-3, weight_decay=5e-4, foreach=False)
    fused = FusedAdamW(b, lr=1e-3, weight_decay=5e-4, max_grad_norm=clip)
    for step in range(4):
        gs = _grads(step, scale)
        for p, q, g in zip(a, b, gs):
            p.grad, q.grad = g.clone(), g.clone()
        if clip is not None:
            want_norm = torch.nn.utils.clip_grad_norm_(a, clip)
        ref.step()
        fused.step()
        if step == 2:                       # lr changes between steps (cosine schedule)
            for grp in ref.param_groups + fused.param_groups:
                grp["lr"] = 5e-4
        torch.cuda.synchronize()
        if clip is not None:
            torch.testing.assert_close(fused.last_grad_norm.cpu()[0], want_norm.cpu(), rtol=1e-5, atol=0)
        for p, q in zip(a, b):
            torch.testing.assert_close(q.detach(), p.detach(), rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(fused.state[q]["exp_avg"], ref.state[p]["exp_avg"], rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(fused.state[q]["exp_avg_sq"], ref.state[p]["exp_avg_sq"], rtol=1e-5, atol=1e-9)
            assert float(fused.state[q]["step"]) == float(ref.state[p]["step"]) == step + 1


def test_fused_adamw_state_dict_interchange():
    """A torch AdamW state resumes in FusedAdamW and the reverse (last.pt interop)."""
    from yolomi.optim import FusedAdamW
    a, b = _params(1), _params(1)
    ref = torch.optim.AdamW(a, lr=1e-3, weight_decay=5e-4, foreach=False)
    for step in range(2):
        for p, g in zip(a, _grads(step, 1.0)):
            p.grad = g
        ref.step()
    with torch.no_grad():
        for p, q in zip(a, b):
            q.copy_(p)
    fused = FusedAdamW(b, lr=1e-3, weight_decay=5e-4)
    fused.load_state_dict(copy.deepcopy(ref.state_dict()))   # (load_state_dict keeps same-device tensors)
    back = torch.optim.AdamW([torch.nn.Parameter(p.detach().clone()) for p in a], lr=1e-3, weight_decay=5e-4,
                             foreach=False)
    for step in range(2, 4):
        gs = _grads(step, 1.0)
        for p, q, g in zip(a, b, gs):
            p.grad, q.grad = g.clone(), g.clone()
        ref.step()
        fused.step()
    torch.cuda.synchronize()
    for p, q in zip(a, b):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=1e-5, atol=1e-6)
    sd = fused.state_dict()
    back.load_state_dict(copy.deepcopy(sd))
    assert set(sd["param_groups"][0]) == set(ref.state_dict()["param_groups"][0])
    assert all(float(back.state[p]["step"]) == 4 for p in back.param_groups[0]["params"])


def test_fused_adamw_in_train_step():
    """The model's flat-buffer gradients feed the fused step; the parameters move as torch's would."""
    from oracle import model as om
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from yolomi.optim import FusedAdamW
    cfg = om.load_cfg("n")
    _, _, P = om.build(cfg)
    m = build_yolo11(cfg, ch=1, nc=5)
    m.load_state_dict(P)
    m = m.cuda().train()
    crit = v8DetectionLoss(m)
    b = {k: v.cuda() for k, v in synth_batch(2, 256, seed=3).items()}
    loss, _ = crit(m(b["img"]), b)
    loss.backward()
    live = [p for p in m.parameters() if p.grad is not None]      # (the frozen DFL projection has none)
    assert len(live) > 200
    shadow = [p.detach().clone().requires_grad_(True) for p in live]
    for s, p in zip(shadow, live):
        s.grad = p.grad.clone()
    ref = torch.optim.AdamW(shadow, lr=1e-3, weight_decay=5e-4, foreach=False)
    torch.nn.utils.clip_grad_norm_(shadow, 10.0)
    ref.step()
    opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=5e-4, max_grad_norm=10.0)
    opt.step()
    torch.cuda.synchronize()
    for s, p in zip(shadow, live):
        torch.testing.assert_close(p.detach(), s.detach(), rtol=1e-5, atol=1e-6)
