"""Concat.forward on standalone tensors (models/yolo11_modules.py:277-285) as device copies.

Within the model plan a concatenation costs nothing (every producer writes its channel slice of
the consumer's buffer, yolomi.graph); this is the module called on its own: each input is one
strided 2-D copy (ym_copy2d: `outer` rows of its inner block) into the output, and the backward
copies the matching blocks of the output gradient back out."""
from __future__ import annotations

import math

import torch

from ._lib import YolomiError, call, require_device, stream_ptr


def _copy_blocks(dst, src_list, d, to_out):
    """to_out: copy each src into its slice of dst along d; else copy dst's slices into each src."""
    outer = math.prod(dst.shape[:d])
    esz = dst.element_size()
    row_out = math.prod(dst.shape[d:]) * esz
    off = 0
    st = stream_ptr(dst.device)
    for t in src_list:
        row = math.prod(t.shape[d:]) * esz
        if to_out:
            call("ym_copy2d", dst.data_ptr() + off, row_out, t.data_ptr(), row, row, outer, st)
        else:
            call("ym_copy2d", t.data_ptr(), row, dst.data_ptr() + off, row_out, row, outer, st)
        off += row


class _ConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, d, *xs):
        shape = list(xs[0].shape)
        shape[d] = sum(x.shape[d] for x in xs)
        out = torch.empty(shape, dtype=xs[0].dtype, device=xs[0].device)
        _copy_blocks(out, xs, d, True)
        ctx.d, ctx.shapes = d, [x.shape for x in xs]
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        outs = [torch.empty(s, dtype=g.dtype, device=g.device) for s in ctx.shapes]
        _copy_blocks(g, outs, ctx.d, False)
        return (None, *outs)


def concat(xs, d=1):
    if not xs:
        raise YolomiError("Concat of an empty list")
    require_device(*xs)
    nd = xs[0].dim()
    d = d % nd
    for x in xs:
        if x.dim() != nd or x.dtype != xs[0].dtype or any(x.shape[i] != xs[0].shape[i] for i in range(nd) if i != d):
            raise YolomiError(f"Concat: incompatible shapes/dtypes {[tuple(t.shape) for t in xs]} along dim {d}")
    return _ConcatFn.apply(d, *[x.contiguous() for x in xs])
