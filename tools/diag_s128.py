"""Diagnostic: s@128 step — GPU vs reference assignment (fg / tgi on each side's heads) and the
parameters furthest from the reference gradient."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd"), str(ROOT / "tests")]
import numpy as np
import torch
from oracle import model as om
from oracle import loss as ol
from models import build_yolo11
from losses import v8DetectionLoss

d = np.load(ROOT / "tests/golden/model_s128.npz")
cfg = om.load_cfg("s")
layers, save, P = om.build(cfg)
m = build_yolo11(cfg, ch=1, nc=5)
m.load_state_dict(P)
m = m.cuda().train()
b = {k: torch.from_numpy(d[k]).cuda() for k in ("img", "batch_idx", "cls", "bboxes")}
cb = {k: torch.from_numpy(d[k]) for k in ("batch_idx", "cls", "bboxes")}
heads = m(b["img"])
gh = [h.detach().cpu().clone() for h in heads]
rh = [torch.from_numpy(d[f"head{i}"]) for i in range(3)]
_, _, ig = ol.v8_loss([h.clone() for h in gh], cb, return_internals=True)
_, _, ir = ol.v8_loss([h.clone() for h in rh], cb, return_internals=True)
print("fg equal", torch.equal(ig["fg"], ir["fg"]), int(ig["fg"].sum()), int(ir["fg"].sum()))
print("tgi equal on fg", torch.equal(ig["tgi"][ir["fg"]], ir["tgi"][ir["fg"]]))
print("target score sum", float(ig["target_scores"].sum()), float(ir["target_scores"].sum()))
for i in range(3):
    print("head", i, float((gh[i] - rh[i]).norm() / rh[i].norm()))
