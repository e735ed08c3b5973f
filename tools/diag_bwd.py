"""Diagnostic: per-parameter gradient error of the plan's backward vs oracle autograd, fixed head grads."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd")]
import torch
from oracle import model as om
from models import build_yolo11
cfg = om.load_cfg("n")
layers, save, P = om.build(cfg)
m = build_yolo11(cfg, ch=1, nc=5)
m.load_state_dict(P)
m = m.cuda().train()
g = torch.Generator().manual_seed(3)
img = torch.rand(2, 1, 256, 256, generator=g)
heads = m(img.cuda())
dh = [torch.randn(h.shape, generator=g) * 0.01 for h in heads]
torch.autograd.backward(heads, [t.cuda() for t in dh])
Q = {k: v.clone() for k, v in P.items()}
leaf = {k: v.requires_grad_(True) for k, v in Q.items()
        if v.is_floating_point() and "running" not in k and not k.endswith("dfl.conv.weight")}
ref = om.forward(Q, layers, save, img, training=True)
torch.autograd.backward(ref, dh)
for k, p in m.named_parameters():
    if not p.requires_grad or not k.endswith("conv.weight"):
        continue
    r = leaf[k].grad
    err = float((p.grad.cpu().double() - r.double()).norm()) / max(float(r.norm()), 1e-12)
    print(f"{k:40s} rel {err:.4f}  |ref| {float(r.norm()):.4g}")
