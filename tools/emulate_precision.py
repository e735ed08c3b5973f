"""Precision model of the HIP training path, emulated in fp32 autograd on the CPU.

Rounds every tensor the HIP path stores in 16 bits (activations and pre-BN conv outputs:
fp16 forward; their gradients: bf16 or fp16 backward) and compares parameter gradients with
the plain fp32 oracle on the network-backward test setup (tests/test_gpu_model.py).  Tells
whether an observed gradient error is explained by storage rounding alone.

usage: python tools/emulate_precision.py [grad dtype: bf16|fp16|fp32]
"""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import model as om  # noqa: E402

GRAD = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[sys.argv[1] if len(sys.argv) > 1 else "bf16"]


class Q(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.half().float()

    @staticmethod
    def backward(ctx, g):
        return g.to(GRAD).float()


LAYERS = None   # restrict the rounding to these model.<i> layers (None: all)


def conv(P, pre, x, s=1, act=True, training=True):
    w = P[pre + ".conv.weight"]
    g = x.shape[1] // w.shape[1]
    on = LAYERS is None or int(pre.split(".")[1]) in LAYERS
    q = Q.apply if on else (lambda t: t)
    y = F.conv2d(q(x), w, None, s, w.shape[-1] // 2, 1, g)
    y = q(y)
    rm, rv = P[pre + ".bn.running_mean"], P[pre + ".bn.running_var"]
    y = F.batch_norm(y, rm, rv, P[pre + ".bn.weight"], P[pre + ".bn.bias"], training, om.BN_MOM, om.BN_EPS)
    if training:
        P[pre + ".bn.num_batches_tracked"] += 1
    return F.silu(y) if act else y


def grads(P, layers, save, img, dh, emulate):
    Q_ = {k: v.clone() for k, v in P.items()}
    leaf = {k: v.requires_grad_(True) for k, v in Q_.items()
            if v.is_floating_point() and "running" not in k and not k.endswith("dfl.conv.weight")}
    saved = om.conv
    if emulate:
        om.conv = conv
    try:
        out = om.forward(Q_, layers, save, img, training=True)
    finally:
        om.conv = saved
    torch.autograd.backward(out, dh)
    return {k: v.grad for k, v in leaf.items()}


def main():
    global LAYERS
    if len(sys.argv) > 2:
        lo, hi = map(int, sys.argv[2].split("-"))
        LAYERS = set(range(lo, hi + 1))
    cfg = om.load_cfg("n")
    layers, save, P = om.build(cfg)
    g = torch.Generator().manual_seed(3)
    img = torch.rand(2, 1, 256, 256, generator=g)
    with torch.no_grad():
        heads = om.forward({k: v.clone() for k, v in P.items()}, layers, save, img, training=True)
    dh = [torch.randn(h.shape, generator=g) * 0.01 for h in heads]
    ref = grads(P, layers, save, img, dh, False)
    emu = grads(P, layers, save, img, dh, True)
    gmax = max(float(v.norm()) for v in ref.values())
    rows = []
    for k, r in ref.items():
        e = float((emu[k] - r).norm()) / max(float(r.norm()), 1e-4 * gmax)
        rows.append((e, k))
    rows.sort()
    for e, k in rows[-12:]:
        print(f"{e:.4f} {k}")


if __name__ == "__main__":
    main()
