"""Per-run checksums of one training step under each executor setting (locates a divergence that
tests/test_gpu_determinism.py reports only as a failed equality).

usage: python tools/det_debug.py
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def step(model, crit, b):
    model.zero_grad(set_to_none=True)
    heads = model(b["img"])
    loss, _ = crit(heads, b)
    loss.backward()
    torch.cuda.synchronize()
    h = torch.cat([x.detach().double().reshape(-1) for x in heads])
    g = [p.grad.detach().double() for p in model.parameters() if p.grad is not None]
    return h, float(loss.detach()), [float(x.sum()) for x in g]


def fmt(r, ref):
    h, loss, gs = r
    dh = float((h - ref[0]).abs().max())
    bad = [i for i, (a, c) in enumerate(zip(gs, ref[2])) if a != c]
    return (f"head_sum={float(h.sum()):.9e} max|dh|={dh:.3e} loss={loss:.9e} "
            f"grads_differ={bad[:12]}{'...' if len(bad) > 12 else ''}")


def main():
    from oracle import model as om
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    cfg = om.load_cfg("n")
    _, _, P = om.build(cfg)
    b = {k: v.cuda() for k, v in synth_batch(4, 320, seed=11).items()}
    m = build_yolo11(cfg, ch=1, nc=5)
    m.load_state_dict(P)
    m = m.cuda().train()
    crit = v8DetectionLoss(m)
    bufs = {k: v.clone() for k, v in m.state_dict().items()}
    ref = None
    os.environ["YM_GRAPH"] = "0"
    for side, streams in (("1", "3"), ("1", "3"), ("0", "3"), ("1", "1"), ("1", "2"), ("0", "2"), ("0", "1"),
                          ("1", "3")):
        os.environ["YM_SIDE_STREAM"], os.environ["YM_STREAMS"] = side, streams
        m.load_state_dict(bufs)
        r = step(m, crit, b)
        ref = ref or r
        print(f"eager side={side} streams={streams}: {fmt(r, ref)}", flush=True)
    for k in ("YM_SIDE_STREAM", "YM_STREAMS", "YM_GRAPH"):
        os.environ.pop(k, None)
    for trial in range(2):
        m2 = build_yolo11(cfg, ch=1, nc=5)
        m2.load_state_dict(P)
        m2 = m2.cuda().train()
        crit2 = v8DetectionLoss(m2)
        for i in range(4):
            m2.load_state_dict(bufs)
            r = step(m2, crit2, b)
            print(f"graph model {trial} step {i}: {fmt(r, ref)}", flush=True)


if __name__ == "__main__":
    main()
