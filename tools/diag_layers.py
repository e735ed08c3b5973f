"""Diagnostic: per-layer forward relative error (GPU plan vs CPU oracle fp32) for n@320 bs2."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd")]
import numpy as np
import torch
from oracle import model as om
from models import build_yolo11

d = np.load(ROOT / "tests/golden/model_n320.npz")
cfg = om.load_cfg("n")
layers, save, P = om.build(cfg)
m = build_yolo11(cfg, ch=1, nc=5)
m.load_state_dict(P)
m = m.cuda().train()
img = torch.from_numpy(d["img"])
heads = m(img.cuda())
plan = m.__dict__["_ym_last_plan"]
allo = []
with torch.no_grad():
    om.forward({k: v.clone() for k, v in P.items()}, layers, save, img, training=True, keep_all=allo)
for i, v in enumerate(plan.layer_outs):
    if v is None:
        continue
    ours = v.act.t[..., v.c0:v.c0 + v.c].float().permute(0, 3, 1, 2).cpu()
    ref = allo[i]
    r = float((ours - ref).norm() / ref.norm())
    print(f"layer {i:2d} {tuple(ref.shape)} rel {r:.4f}")
for i in range(3):
    r = float((heads[i].detach().cpu() - allo[-1][i]).norm() / allo[-1][i].norm())
    box = float((heads[i].detach().cpu()[:, :64] - allo[-1][i][:, :64]).norm() / allo[-1][i][:, :64].norm())
    cls = float((heads[i].detach().cpu()[:, 64:] - allo[-1][i][:, 64:]).norm() / allo[-1][i][:, 64:].norm())
    print(f"head {i} rel {r:.4f} box {box:.4f} cls {cls:.5f}")
