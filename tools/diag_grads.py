"""Diagnostic: per-parameter grad-norm ratio (GPU plan / reference golden) for the n@320 step."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd"), str(ROOT / "tests")]
import numpy as np
import torch
from oracle import model as om
from models import build_yolo11
from losses import v8DetectionLoss

d = np.load(ROOT / "tests/golden/model_n320.npz")
cfg = om.load_cfg("n")
layers, save, P = om.build(cfg)
m = build_yolo11(cfg, ch=1, nc=5)
m.load_state_dict(P)
m = m.cuda().train()
b = {k: torch.from_numpy(d[k]).cuda() for k in ("img", "batch_idx", "cls", "bboxes")}
heads = m(b["img"])
crit = v8DetectionLoss(m)
loss, items = crit(heads, b)
print("loss", float(loss), float(d["loss"][0]), "items", items.tolist(), d["items"].tolist())
loss.backward()
ref = dict(zip(d["grad_names"], d["grad_norm"]))
for k, p in m.named_parameters():
    if p.requires_grad:
        print(f"{k:45s} {float(p.grad.norm()) / max(ref[k], 1e-12):7.3f}  ref {ref[k]:.4g}")
