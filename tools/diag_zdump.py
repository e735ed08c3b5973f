"""Diagnostic: dump every ConvBN's forward z (pre-BN conv output) and BN scale/shift of the s@128
step to a file (argv[1]); with argv[2] also compare against an earlier dump, op by op."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd"), str(ROOT / "tests")]
import numpy as np
import torch
from test_gpu_model import _batch, _seeded_model
from yolomi.graph import ConvBN
from yolomi._lib import lib
import ctypes

d = np.load(ROOT / "tests/golden/model_s128.npz")
m = _seeded_model("s").train()
batch = _batch(d)
heads = m(batch["img"])
torch.cuda.synchronize()
plan = m.__dict__["_ym_last_plan"]
out = {}
for i, op in enumerate(plan.ops):
    if type(op) is ConvBN:
        algo = lib().ym_conv_algo(ctypes.byref(op.desc), 0) if hasattr(op, "desc") else -1
        out[i] = (op.z.float().cpu().clone(), op.bnv.cpu().clone(), algo, type(op).__name__,
                  (op.ci, op.co, op.k, op.s, op.y.H, op.y.W, getattr(op.x, "ld", 0), getattr(op.x, "c0", 0)))
torch.save(out, sys.argv[1])
if len(sys.argv) > 2:
    ref = torch.load(sys.argv[2])
    for i, (z, bnv, algo, nm, geo) in out.items():
        z0, b0 = ref[i][0], ref[i][1]
        dz = float((z - z0).abs().max() / z0.abs().max().clamp_min(1e-12))
        db = float((bnv - b0).abs().max() / b0.abs().max().clamp_min(1e-12))
        flag = " <<<" if dz > 1e-3 or db > 1e-3 else ""
        print(f"op {i:3d} {nm:10s} algo {algo} geo {geo} z {dz:.2e} bn {db:.2e}{flag}")
