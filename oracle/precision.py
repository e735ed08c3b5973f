"""TEST ORACLE ONLY — the HIP path's 16-bit storage policy applied to the fp32 oracle.

Imported by tests/ only.  The HIP training path keeps activations and pre-BatchNorm conv
outputs in fp16 and their gradients in bf16 (DESIGN.md §dtype policy); every Conv block of the
oracle (oracle/model.py:conv, restating yolo11_modules.py:21-33) is wrapped so that its input
and its conv output are rounded exactly there: fp16 in the forward, bf16 in the backward.

Why the tests need it: training-mode YOLOv11 backbones are discontinuous in their inputs
through SPPF's 5x5 max-pools (yolo11_modules.py:92-105) — the pool gradient goes to the
window's first maximum, and a 2^-11 rounding of the backbone activations moves the argmax of
near-tied windows.  Measured with tools/emulate_precision.py on the network-backward case: the
fp32 oracle against fp32-vs-fp64 differs by <= 4e-5, but rounding ONLY layers 0-8 to fp16
storage moves backbone BatchNorm gradients by up to 17% (layers 9 / 10 / 11-23 alone: 2.4% /
0.45% / 0.42%), with bf16 and fp16 gradient storage alike.  A gradient parity bound for
backbone parameters is therefore stated relative to this rounding model's own distance from
the fp32 reference, not as a fixed number.
"""
from __future__ import annotations

from contextlib import contextmanager

import torch
import torch.nn.functional as F

from . import model as om


class _Round(torch.autograd.Function):
    grad_dtype = torch.bfloat16

    @staticmethod
    def forward(ctx, x):
        return x.half().float()

    @staticmethod
    def backward(ctx, g):
        return g.to(_Round.grad_dtype).float()


def _conv_rounded(P, pre, x, s=1, act=True, training=True):
    """oracle.model.conv with the HIP path's storage points rounded."""
    w = P[pre + ".conv.weight"]
    g = x.shape[1] // w.shape[1]
    y = F.conv2d(_Round.apply(x), w, None, s, w.shape[-1] // 2, 1, g)
    y = _Round.apply(y)
    rm, rv = P[pre + ".bn.running_mean"], P[pre + ".bn.running_var"]
    y = F.batch_norm(y, rm, rv, P[pre + ".bn.weight"], P[pre + ".bn.bias"], training, om.BN_MOM, om.BN_EPS)
    if training:
        P[pre + ".bn.num_batches_tracked"] += 1
    return F.silu(y) if act else y


@contextmanager
def hip_storage_rounding(grad_dtype=torch.bfloat16):
    """Within the block, oracle.model.forward rounds like the HIP path stores."""
    saved, saved_dt = om.conv, _Round.grad_dtype
    om.conv, _Round.grad_dtype = _conv_rounded, grad_dtype
    try:
        yield
    finally:
        om.conv, _Round.grad_dtype = saved, saved_dt
