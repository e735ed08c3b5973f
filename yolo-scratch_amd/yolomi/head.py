"""Detect-head views and the eval-mode decode (Detect.inference) on the GPU."""
from __future__ import annotations

import ctypes

import torch

from ._lib import YolomiError, call, stream_ptr


def _levels(level_hw):
    nl = len(level_hw)
    lh = (ctypes.c_int * nl)(*[h for h, _ in level_hw])
    lw = (ctypes.c_int * nl)(*[w for _, w in level_hw])
    return nl, lh, lw


def level_views(head: torch.Tensor, level_hw):
    """(B, A, no) head buffer -> [(B, no, h, w)] per level, as the reference's Detect returns (:239-246).

    Each view keeps a reference to the whole buffer (`_ym_head`) so the loss consumes the
    buffer directly instead of re-concatenating the levels."""
    B, A, no = head.shape
    out, off = [], 0
    for h, w in level_hw:
        v = head[:, off:off + h * w, :].view(B, h, w, no).permute(0, 3, 1, 2)
        v._ym_head = head
        v._ym_levels = tuple(level_hw)
        out.append(v)
        off += h * w
    return out


def inference(detect, head: torch.Tensor, level_hw) -> torch.Tensor:
    """y (B, 4+nc, A): xywh*stride via the DFL projection with the module's (random, Q5) weights."""
    B, A, no = head.shape
    nc = no - 64
    nl, lh, lw = _levels(level_hw)
    strides = (ctypes.c_float * nl)(*[float(s) for s in detect.stride])
    dflw = detect.dfl.conv.weight.detach().reshape(-1).float().contiguous()
    y = torch.empty(B, 4 + nc, A, dtype=torch.float32, device=head.device)
    call("ym_detect_decode", head.data_ptr(), B, A, nc, nl, lh, lw, strides, dflw.data_ptr(), y.data_ptr(),
         stream_ptr(head.device))
    return y


class _DFLFn(torch.autograd.Function):
    """DFL.forward as one autograd node: ym_dfl_fwd / ym_dfl_bwd (fp32, the conv weight frozen)."""

    @staticmethod
    def forward(ctx, x, w, c1):
        B, _, A = x.shape
        y = torch.empty(B, 4, A, dtype=torch.float32, device=x.device)
        call("ym_dfl_fwd", x.data_ptr(), B, A, c1, w.data_ptr(), y.data_ptr(), stream_ptr(x.device))
        ctx.save_for_backward(x, w)
        ctx.c1 = c1
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        B, _, A = x.shape
        dy = dy.float().contiguous()
        dx = torch.empty_like(x)
        call("ym_dfl_bwd", x.data_ptr(), B, A, ctx.c1, w.data_ptr(), dy.data_ptr(), dx.data_ptr(),
             stream_ptr(x.device))
        return dx, None, None


def dfl(x: torch.Tensor, weight: torch.Tensor, c1: int) -> torch.Tensor:
    """DFL.forward (yolo11_modules.py:189-192) on the GPU: x (b, 4*c1, a) -> (b, 4, a)."""
    if not x.is_cuda:
        raise YolomiError("yolomi kernels run on the MI355X only (got a CPU tensor)")
    b, c, a = x.shape
    if c != 4 * c1:
        raise YolomiError(f"DFL expects 4*c1={4 * c1} channels, got {c}")
    w = weight.detach().reshape(-1).float().contiguous()
    xf = x.float().contiguous()
    if torch.is_grad_enabled() and x.requires_grad:
        return _DFLFn.apply(xf, w, c1)
    y = torch.empty(b, 4, a, dtype=torch.float32, device=x.device)
    call("ym_dfl_fwd", xf.data_ptr(), b, a, c1, w.data_ptr(), y.data_ptr(), stream_ptr(x.device))
    return y
