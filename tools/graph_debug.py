"""Capture the model plan's forward as a HIP graph under different stream settings (debugging)."""
import os
import sys
import faulthandler
faulthandler.enable()
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, R)
sys.path.insert(0, R + "/yolo-scratch_amd")
import torch
from oracle import model as om
from models import build_yolo11
from datasets.synthetic import synth_batch
cfg = om.load_cfg("n")
m = build_yolo11(cfg, ch=1, nc=5).cuda().train()
b = synth_batch(2, 256, seed=1)
img = b["img"].cuda()
mode = sys.argv[1]
if mode == "prefix":
    # capture only the first N forward ops of the plan on YM_STREAMS scheduler streams (bisecting a crash)
    n_ops = int(sys.argv[2])
    with torch.no_grad():
        m(img)
    torch.cuda.synchronize()
    plan = m.__dict__["_ym_last_plan"]
    ops = plan.ops[:n_ops]
    print("ops", len(plan.ops), "capturing", len(ops), "streams", plan._nstreams(), flush=True)
    sched, need = plan._schedule(ops, "fwd", plan._nstreams())
    for i in range(len(ops)):
        op = ops[i]
        print(i, type(op).__name__, getattr(getattr(op, "m", None), "__class__", type(None)).__name__,
              "stream", sched[i][0], "waits", sched[i][1], "rec" if i in need else "", flush=True)
    plan._run(ops, "fwd")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        plan._run(ops, "fwd")
    g.replay()
    torch.cuda.synchronize()
    print("prefix", n_ops, "captured and replayed", flush=True)
elif mode == "raw":
    # minimal: capture one ctypes launch
    from yolomi._lib import call
    from yolomi.graph import run_model
    with torch.no_grad():
        m(img)
    plan = m.__dict__["_ym_last_plan"]
    op = plan.ops[1]
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        print("capture stream", torch.cuda.current_stream().cuda_stream, flush=True)
        op.forward(plan, torch.cuda.current_stream().cuda_stream)
    print("captured one op", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("replayed", flush=True)
else:
    from losses import v8DetectionLoss
    crit = v8DetectionLoss(m)
    bb = {k: v.cuda() for k, v in b.items()}
    for i in range(3):
        h = m(img)
        torch.cuda.synchronize()
        print("fwd", i, "ok", flush=True)
        loss, _ = crit(h, bb)
        loss.backward()
        torch.cuda.synchronize()
        print("bwd", i, "ok", float(loss), flush=True)
