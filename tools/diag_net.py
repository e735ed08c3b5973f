"""Diagnostic: s@128 (model_s128.npz) training step — every parameter's gradient error against the
fp32 oracle's backward at the GPU's own head gradients, relative to the storage-rounding model's
error (the quantity test_gpu_network.check_network bounds by 1).  Prints the worst ratios; run under
different YM_* toggles to find which kernel path moves the error."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd"), str(ROOT / "tests")]
import numpy as np
import torch
from oracle import loss as ol
from test_gpu_model import _batch, _seeded_model
from test_gpu_network import _oracle_grads
from losses import v8DetectionLoss

d = np.load(ROOT / "tests/golden/model_s128.npz")
m = _seeded_model("s").train()
batch = _batch(d)
heads = m(batch["img"])
loss, items = v8DetectionLoss(m)(heads, batch)
loss.backward()
cb = {k: v.cpu() for k, v in batch.items() if k != "img"}
hg = [h.detach().cpu().clone().requires_grad_(True) for h in heads]
ol.v8_loss(hg, cb)[0].backward()
dh = [h.grad for h in hg]
at = _oracle_grads("s", d["img"], dh)
emu = _oracle_grads("s", d["img"], dh, rounding=True)
gmax = max(float(v.norm()) for v in at.values())
rows = []
for k, p in m.named_parameters():
    if not p.requires_grad:
        continue
    r = at[k].double()
    sc = max(float(r.norm()), 1e-4 * gmax)
    e1 = float((p.grad.cpu().double() - r).norm()) / sc
    ee = float((emu[k].double() - r).norm()) / sc
    rows.append((e1 / max(3e-2, 2 * ee), k, e1, ee))
rows.sort()
for row in rows[-12:]:
    print("%.3f %-40s err %.4f emu %.4f" % row)
