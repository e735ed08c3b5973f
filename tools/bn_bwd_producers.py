"""Who writes each BatchNorm layer's output gradient dy, in backward order (CPU only: builds the plan on CPU).

For every ConvBN L of the s@640 plan: the ops that write a gradient range overlapping L.y, in the order the backward
runs them, whether the LAST of them is a ConvBN data gradient whose input view is exactly L.y (the case where that
launch's epilogue holds the complete dy of L and could form L's BatchNorm-backward statistics), and which dgrad
kernel that launch runs at the bench's batch.  The per-layer BN reduce time column comes from a bn_bench.txt.

usage: python tools/bn_bwd_producers.py [--scale s --imgsz 640 --batch 64 --bn profiles/r04/at_8019a42/bn_bench.txt]
"""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)

ALGO = {0: "gemm", 1: "halo", 2: "pipe", 3: "direct", 4: "hpipe"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="s")
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--bn", default=str(ROOT / "profiles/r04/at_8019a42/bn_bench.txt"))
    args = ap.parse_args()
    import torch
    import yaml
    from models import build_yolo11
    from yolomi._lib import lib
    from yolomi import graph as G

    red = {}
    try:
        for line in Path(args.bn).read_text().splitlines():
            f = line.split()
            if f and f[0].isdigit():
                red[int(f[0])] = float(f[8])
    except OSError:
        pass
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = args.scale
    model = build_yolo11(cfg, ch=1, nc=5).train()
    plan = G.Plan(model, args.batch, args.imgsz, args.imgsz, torch.device("cpu"), True)
    plan.input_requires_grad = False
    plan.is_model = True
    G.lower_model(plan, model, (args.batch, args.imgsz, args.imgsz))
    ops = plan.ops
    idx = {id(op): i for i, op in enumerate(ops)}
    writers = []                     # (op index, gradient key) in backward order
    fused_us = other_us = 0.0
    print(f"{'op':>4} {'C':>4} {'map':>7} | writers of dy (bwd order)           | last writer -> fusable kernel | reduce us")
    for op in reversed(ops):
        i = idx[id(op)]
        if type(op) in (G.ConvBN, G.StemConvBN) or isinstance(op, G.ConvBN):
            key = G._kg(op.y)
            ws = [(j, k) for j, k in writers if G._overlap(key, k)]
            last = ws[-1][0] if ws else None
            verdict = "-"
            if last is not None:
                P = ops[last]
                if type(P) is G.ConvBN and P.x.act is op.y.act and P.x.c0 == op.y.c0 and P.x.c == op.y.c:
                    verdict = f"op {last} dgrad {ALGO.get(lib().ym_conv_algo(ctypes.byref(P.desc), 1), '?')}"
                else:
                    verdict = f"no ({type(P).__name__} {last})"
            us = red.get(i, 0.0)
            if verdict.startswith("op"):
                fused_us += us
            else:
                other_us += us
            print(f"{i:4d} {op.co:4d} {op.y.H:3d}x{op.y.W:<3d} | {str([j for j, _ in ws]):35s} | {verdict:29s} | {us:6.1f}")
        R, W = op.rw(plan, "bwd")
        Rset = set(R)
        for k in W:
            if k[0] == "g" and k not in Rset:
                writers.append((i, k))
        if isinstance(op, G.ConvBN) and type(op) is not G.StemConvBN and op.x is not None and plan.needs_grad(op.x):
            writers.append((i, G._kg(op.x)))
    print(f"reduce us on fusable layers {fused_us:.0f}, elsewhere {other_us:.0f}")


if __name__ == "__main__":
    main()
