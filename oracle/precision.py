"""TEST ORACLE ONLY — the HIP path's 16-bit storage policy applied to the fp32 oracle.

Imported by tests/ only.  The HIP training path keeps activations and pre-BatchNorm conv
outputs in fp16 and their gradients in bf16 (DESIGN.md §dtype policy); every Conv block of the
oracle (oracle/model.py:conv, restating yolo11_modules.py:21-33) is wrapped so that its input
and its conv output are rounded exactly there: fp16 in the forward, bf16 in the backward; the conv's
weights are the fp16 (forward) / bf16 (data gradient) copies the kernels read (_ConvQ).

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


_jitter = {"gen": None}


class _ConvQ(torch.autograd.Function):
    """conv2d with the HIP path's operand dtypes: the forward multiplies fp16 activations by the
    fp16 forward weight copy, the data gradient uses the bf16 transposed weight copy, and the
    weight gradient reads the fp16 activations converted to bf16 at staging (prep_weights_kernel,
    conv_gemm / wgrad kernels).  x arrives already rounded to fp16 (_Round)."""

    @staticmethod
    def forward(ctx, x, w, s, g):
        ctx.save_for_backward(x, w)
        ctx.s, ctx.g = s, g
        return F.conv2d(x, w.half().float(), None, s, w.shape[-1] // 2, 1, g)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        s, g, p = ctx.s, ctx.g, w.shape[-1] // 2
        dx = torch.nn.grad.conv2d_input(x.shape, w.bfloat16().float(), gy, s, p, 1, g)
        dw = torch.nn.grad.conv2d_weight(x.bfloat16().float(), w.shape, gy, s, p, 1, g)
        return dx, dw, None, None


def _conv_rounded(P, pre, x, s=1, act=True, training=True):
    """oracle.model.conv with the HIP path's storage points rounded (and, for a jittered sample, the
    fp32 conv output moved by <= 2^-20 relative per element before its fp16 rounding: the order of the
    accumulation-order differences between the GPU's MFMA sums and torch's)."""
    w = P[pre + ".conv.weight"]
    g = x.shape[1] // w.shape[1]
    y = _ConvQ.apply(_Round.apply(x), w, s, g)
    if _jitter["gen"] is not None:
        u = torch.rand(y.shape, generator=_jitter["gen"], dtype=y.dtype) * 2 - 1
        y = y * (1 + u * 2.0 ** -20)
    y = _Round.apply(y)
    rm, rv = P[pre + ".bn.running_mean"], P[pre + ".bn.running_var"]
    y = F.batch_norm(y, rm, rv, P[pre + ".bn.weight"], P[pre + ".bn.bias"], training, om.BN_MOM, om.BN_EPS)
    if training:
        P[pre + ".bn.num_batches_tracked"] += 1
    return F.silu(y) if act else y


@contextmanager
def hip_storage_rounding(grad_dtype=torch.bfloat16, jitter=0):
    """Within the block, oracle.model.forward rounds like the HIP path stores.

    jitter > 0 draws sample `jitter` of the rounding model: the same storage rounding after a seeded
    per-element fp32-level perturbation of every conv output.  The network is chaotic in these
    last-bit differences (SPPF argmax routing, fp16 rounding flips that the BatchNorm layers
    renormalise and pass on), so the GPU path's gradient is ONE draw from the distribution these
    samples span; parity bounds built on the rounding model take the worst of a few samples."""
    saved, saved_dt = om.conv, _Round.grad_dtype
    om.conv, _Round.grad_dtype = _conv_rounded, grad_dtype
    _jitter["gen"] = torch.Generator().manual_seed(1000 + jitter) if jitter else None
    try:
        yield
    finally:
        om.conv, _Round.grad_dtype = saved, saved_dt
        _jitter["gen"] = None
