"""NHWC execution plan for the YOLOv11 module tree on MI355X.

A module (the whole YOLOv11 or any building block: Conv, C3k2, SPPF, C2PSA,
Detect ...) is lowered ONCE per input shape into a flat list of ops over
preallocated NHWC activation buffers (fp16; gradients bf16).  Concatenations and splits of the
reference (yolo11_modules.py C2f:59-63, C3k:78, SPPF:104-105, PSA:156-159,
C2PSA:175-177, Concat:284-285, yaml head rows) become channel slices: every
producer writes straight into its slice of the consumer's buffer.  Forward
runs the ops in order; backward runs them in reverse over a mirrored set of
gradient buffers, deciding per slice whether to overwrite or accumulate.

Every arithmetic step is a libyolomi kernel; this file only plans buffers and
launches.  Parameter gradients land in one flat fp32 buffer per plan
(`Plan.grad_flat`), with each parameter's `.grad` a view of it, so the
data-parallel all-reduce is one RCCL call.
"""
from __future__ import annotations

import ctypes
import math
import os
import weakref

import numpy as np
import torch

from ._lib import BnEvalEntry, BnFold, ConvDesc, WPrepEntry, YolomiError, call, lib, stream_ptr

BF16 = torch.bfloat16
F16 = torch.float16
F32 = torch.float32
ACT_DTYPE, GRAD_DTYPE = F16, BF16      # activations fp16 (precision), gradients bf16 (range)
BN_EPS, BN_MOM = 1e-3, 0.03


# ----------------------------------------------------------------------------- buffers
class Act:
    """One NHWC activation buffer (B, H, W, C) and its gradient mirror."""

    def __init__(self, plan, C, H, W, dtype=ACT_DTYPE, name=""):
        self.plan, self.C, self.H, self.W, self.dtype, self.name = plan, C, H, W, dtype, name
        self.t = torch.empty(plan.B, H, W, C, dtype=dtype, device=plan.dev)
        self.g = None
        self.written = np.zeros(C, bool)
        plan.acts.append(self)

    @property
    def bs(self):
        return self.H * self.W * self.C

    @property
    def M(self):
        return self.plan.B * self.H * self.W

    def grad(self):
        if self.g is None:
            self.g = torch.empty(self.t.shape, dtype=GRAD_DTYPE, device=self.t.device)
        return self.g


class View:
    """Channel slice [c0, c0+c) of an Act."""

    def __init__(self, act: Act, c0: int = 0, c: int | None = None):
        self.act, self.c0 = act, c0
        self.c = act.C - c0 if c is None else c

    def sub(self, c0, c):
        return View(self.act, self.c0 + c0, c)

    @property
    def H(self):
        return self.act.H

    @property
    def W(self):
        return self.act.W

    @property
    def bs(self):
        return self.act.bs

    @property
    def ld(self):
        return self.act.C

    @property
    def M(self):
        return self.act.M

    def ptr(self):
        return self.act.t.data_ptr() + self.c0 * self.act.t.element_size()

    def gptr(self):
        g = self.act.grad()
        return g.data_ptr() + self.c0 * g.element_size()

    # --- gradient bookkeeping (backward)
    def grad_for_write(self, st):
        """Accumulate flag for writing this slice's gradient; zero-fills a partially written slice."""
        w = self.act.written[self.c0:self.c0 + self.c]
        if w.all():
            return 1
        if w.any():
            call("ym_view_axpy", None, 0, 0, self.gptr(), self.bs, self.ld, self.M, self.c, self.H * self.W, 0, 0, st)
            self.act.written[self.c0:self.c0 + self.c] = True
            return 1
        return 0

    def mark(self):
        self.act.written[self.c0:self.c0 + self.c] = True

    def grad_for_read(self, st):
        """Gradient of this slice, zero-filled where no consumer wrote it."""
        if not self.act.written[self.c0:self.c0 + self.c].all():
            acc = self.grad_for_write(st)
            if not acc:
                call("ym_view_axpy", None, 0, 0, self.gptr(), self.bs, self.ld, self.M, self.c, self.H * self.W, 0, 0, st)
            self.mark()
        return self.gptr()


# ----------------------------------------------------------------------------- weights
class WeightStore:
    """bf16 copies of every conv weight of a plan in the two kernel layouts."""

    def __init__(self, plan):
        self.plan = plan
        self.items = []          # (module_param, fwd tensor, t tensor, cout_t)
        self.table_dev = None
        self.key = None

    def add(self, w: torch.nn.Parameter, need_t: bool, cout_t: int | None = None):
        co, ci, kh, kw = w.shape
        cout_t = cout_t or co
        # an eval-mode model plan never runs a backward: no transposed data-gradient copy to prepare
        need_t = need_t and (self.plan.training or not getattr(self.plan, "is_model", False))
        fwd = torch.empty(co, kh, kw, ci, dtype=F16, device=self.plan.dev)
        t = torch.zeros(ci, kh, kw, cout_t, dtype=BF16, device=self.plan.dev) if need_t else None
        self.items.append((w, fwd, t, cout_t))
        return fwd, t

    def refresh(self, st):
        """One launch converting every fp32 OIHW master weight (after each optimizer step)."""
        if not self.items:
            return
        key = tuple(w.data_ptr() for w, *_ in self.items)
        if key != self.key:
            arr = (WPrepEntry * len(self.items))()
            off = 0
            for e, (w, fwd, t, cout_t) in zip(arr, self.items):
                co, ci, kh, kw = w.shape
                e.src, e.dst_fwd, e.dst_t = w.data_ptr(), fwd.data_ptr(), (t.data_ptr() if t is not None else None)
                e.elem_offset, e.cout, e.cin, e.kh, e.kw, e.cout_t = off, co, ci, kh, kw, cout_t
                off += w.numel()
            raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            self.table_dev = raw.to(self.plan.dev)
            self.total = off
            self.key = key
        # no transposed copy in the table (an eval plan): the forward-only launch
        fwd_only = all(t is None for _, _, t, _ in self.items)
        call("ym_prep_weights_fwd" if fwd_only else "ym_prep_weights", self.table_dev.data_ptr(), len(self.items),
             self.total, st)


# ----------------------------------------------------------------------------- ops
def _p(t):
    return None if t is None else t.data_ptr()


# buffer-range keys for the stream scheduler: ('a' activation | 'g' gradient, Act id, c0, c1)
def _ka(v):
    return ("a", id(v.act), v.c0, v.c0 + v.c)


def _kg(v):
    return ("g", id(v.act), v.c0, v.c0 + v.c)


def _overlap(k1, k2):
    if k1[0] != k2[0] or k1[1] != k2[1]:
        return False
    if len(k1) == 2:
        return True
    return k1[2] < k2[3] and k2[2] < k1[3]


class ConvBN:
    """Conv2d (k in {1,3}, groups=1) -> BatchNorm2d -> SiLU|Identity (+ residual) — reference Conv :21-33."""

    def __init__(self, plan, m, x: View, y: View, s=1, act=True, res: View | None = None):
        w = m.conv.weight
        self.m, self.x, self.y, self.res, self.act = m, x, y, res, int(act)
        co, ci, k, _ = w.shape
        assert ci == x.c and co == y.c, (m, ci, x.c, co, y.c)
        self.k, self.s, self.co, self.ci = k, s, co, ci
        oh, ow = (x.H + 2 * (k // 2) - k) // s + 1, (x.W + 2 * (k // 2) - k) // s + 1
        assert (oh, ow) == (y.H, y.W), ((oh, ow), (y.H, y.W))
        B = plan.B
        self.M, self.HW = B * oh * ow, oh * ow
        self.z = torch.empty(self.M, co, dtype=BF16, device=plan.dev)
        self.wf, self.wt = plan.weights.add(w, need_t=x.act is not None)
        d = ConvDesc()
        d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout = B, x.H, x.W, ci, oh, ow, co
        d.k, d.stride, d.pad = k, s, k // 2
        d.x_bs, d.x_ld, d.y_bs, d.y_ld = x.bs, x.ld, self.HW * co, co
        d.out_f32 = 2                                                   # fp16 pre-BN z
        self.desc = d
        self.G = lib().ym_conv_fwd_stat_rows(ctypes.byref(d))
        self.ps = torch.empty(2, max(self.G, lib().ym_bn_bwd_blocks(self.M, co)), co, dtype=F32, device=plan.dev)
        self.bnv = torch.empty(4, co, dtype=F32, device=plan.dev)      # scale, shift, mean, rstd
        self.coef = torch.empty(3, co, dtype=F32, device=plan.dev)
        plan.need_wgrad_ws(d)

    def flops(self):
        return 2 * self.M * self.co * self.ci * self.k * self.k

    def rw(self, plan, phase):
        """(reads, writes) buffer ranges of this op's forward / backward (stream scheduler)."""
        if phase == "fwd":
            return [_ka(self.x)] + ([_ka(self.res)] if self.res else []), [_ka(self.y)]
        w = [_kg(self.y)] + ([_kg(self.x)] if plan.needs_grad(self.x) else []) + ([_kg(self.res)] if self.res else [])
        return [_ka(self.x), _kg(self.y)], w

    def _timed(self, plan, kind, stream, fn, work=None):
        """Run one launch; the bench brackets it with HIP events on its own stream when it times this
        op (plan.probe) or this kernel family (plan.family_events: conv 'fwd' / 'dgrad' / 'wgrad' with
        their algorithmic FLOPs, 'bn' with its algorithmic HBM bytes in `work`)."""
        fam = plan.family_events
        probe = kind == "fwd" and plan.probe is self
        if not probe and (fam is None or kind not in fam):
            fn()
            return
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        fn()
        ev1.record(stream)
        if probe:
            plan.probe_events.append((ev0, ev1))
        if fam is not None and kind in fam:
            ent = (ev0, ev1, self.flops() if work is None else work)
            fam[kind].append(ent)
            if kind != "bn" and self.k == 3 and f"{kind}3" in fam:     # the dense 3x3 convs on their own
                fam[f"{kind}3"].append(ent)

    def _static_args(self, plan):
        """Pointer arguments of this op's forward launches that never change for its plan (the plan's
        own buffers), converted once: at bs1 the eval forward is host-bound and re-deriving them per
        launch (tensor indexing, view offsets) was about half of its ~20 us of host time per conv block.
        Parameters stay looked up per call (a replaced nn.Parameter is seen)."""
        a = self.__dict__.get("_sa")
        if a is None:
            r = self.res
            bnv = tuple(self.bnv[i].data_ptr() for i in range(4))
            ss, sq = self.ps[0].data_ptr(), self.ps[1].data_ptr()
            apply = (self.z.data_ptr(), self.M, self.co, self.HW, bnv[0], bnv[1], self.act,
                     r.ptr() if r else None, r.bs if r else 0, r.ld if r else 0, self.y.ptr(), self.y.bs, self.y.ld,
                     _p(getattr(self, "out32", None)))
            a = self._sa = (bnv, ss, sq, apply)
        return a

    def _fused(self, plan):
        """Whether the training forward runs ym_conv_fwd_bn with the BatchNorm finalize folded into the conv
        launch's tail (the pipelined forward; YM_FOLD=0: conv, then ym_bn_finalize, as for the other kernels)."""
        if os.environ.get("YM_FOLD", "1") == "0":
            return False
        f = self.__dict__.get("_fused_c")
        if f is None:
            f = self._fused_c = bool(lib().ym_conv_fwd_bn_fused(ctypes.byref(self.desc)))
        return f

    def _fold(self, plan):
        """ym_bn_fold argument of this layer; the BatchNorm parameters are looked up per call (a replaced
        Parameter or buffer is seen), the struct rebuilt only when one of them changed."""
        bn = self.m.bn
        (sc, sh, mu, rs), _, _, _ = self._static_args(plan)
        key = (_p(bn.weight), _p(bn.bias), _p(bn.running_mean), _p(bn.running_var), _p(bn.num_batches_tracked),
               plan.bn_ws.data_ptr(), float(bn.momentum), float(bn.eps))
        f = self.__dict__.get("_fold_s")
        if f is None or f[0] != key:
            fs = BnFold(gamma=key[0], beta=key[1], running_mean=key[2], running_var=key[3],
                        num_batches_tracked=key[4], scale=sc, shift=sh, mean=mu, rstd=rs, workspace=key[5],
                        count=float(self.M), momentum=key[6], eps=key[7])
            f = self._fold_s = (key, fs, ctypes.byref(fs))
        return f[2]

    def _bn_fwd(self, plan, st, ss, sq, finalize=True):
        """BatchNorm finalize + apply (+ SiLU, + residual) of the forward: 'bn' family, algorithmic bytes
        = the partial rows read + z read + y written (+ residual read).  finalize=False: the conv launch
        already folded the statistics (ym_conv_fwd_bn), only the apply pass runs here."""
        bn = self.m.bn
        (sc, sh, mu, rs), ssp, sqp, apply = self._static_args(plan)
        r = self.res
        e = self.M * self.co * 2
        work = 8 * self.G * self.co * (1 if plan.training and finalize else 0) + 2 * e + (e if r else 0)

        def run():
            if plan.training and not finalize:
                pass
            elif plan.training:
                call("ym_bn_finalize", ssp, sqp, self.G, self.co, float(self.M), _p(bn.weight),
                     _p(bn.bias), _p(bn.running_mean), _p(bn.running_var), _p(bn.num_batches_tracked),
                     float(bn.momentum), float(bn.eps), sc, sh, mu, rs, plan.bn_ws.data_ptr(), st)
            elif not plan.eval_coeff_batched:
                call("ym_bn_eval_coeff", self.co, _p(bn.weight), _p(bn.bias), _p(bn.running_mean),
                     _p(bn.running_var), float(bn.eps), sc, sh, st)
            call("ym_bn_apply", *apply, st)
        self._timed(plan, "bn", plan._cur_stream, run, work)

    def _eval_one_launch(self, plan):
        """ym_conv_fwd_eval arguments for this op's eval forward (conv + eval BatchNorm + SiLU + residual in one
        launch), or None: the selected kernel has no eval epilogue, a view is misaligned, or SPPF's pools need the
        fp32 copy.  YM_EVAL_FUSE=0 opts out."""
        # keyed on the library's policy generation too: ym_conv_fwd_eval_ok and the K-split workspace are answers of the
        # selection policies in force (yolomi_experimental.h), re-asked after any setter call
        on = (os.environ.get("YM_EVAL_FUSE", "1") != "0" and "out32" not in self.__dict__, lib().ym_policy_generation())
        f = self.__dict__.get("_evf")
        if f is None or f[0] != on:
            args = None
            r = self.res
            if on[0] and (r is None or (r.ptr() % 8 == 0 and r.ld % 4 == 0)) and self.y.ptr() % 16 == 0:
                d = ConvDesc.from_buffer_copy(self.desc)
                d.y_bs, d.y_ld, d.out_f32, d.accumulate = self.y.bs, self.y.ld, 2, 0
                if lib().ym_conv_fwd_eval_ok(ctypes.byref(d)):
                    (sc, sh, _, _), _, _, _ = self._static_args(plan)
                    # the small-grid K-split's fp32 slices: this op's own buffer (ops of a plan may run on side streams)
                    nws = lib().ym_conv_fwd_eval_workspace_size(ctypes.byref(d))
                    self._evws = torch.empty(nws, dtype=torch.uint8, device=plan.dev) if nws else None
                    args = (d, ctypes.byref(d), self.x.ptr(), self.wf.data_ptr(), sc, sh, self.act,
                            r.ptr() if r is not None else None, r.bs if r is not None else 0,
                            r.ld if r is not None else 0, self.y.ptr(),
                            self._evws.data_ptr() if nws else None, nws)
            f = self._evf = (on, args)
        return f[1]

    def forward(self, plan, st):
        if not plan.training:
            ev = self._eval_one_launch(plan)
            if ev is not None:
                bn = self.m.bn
                if not plan.eval_coeff_batched:
                    sc, sh = ev[4], ev[5]
                    call("ym_bn_eval_coeff", self.co, _p(bn.weight), _p(bn.bias), _p(bn.running_mean),
                         _p(bn.running_var), float(bn.eps), sc, sh, st)
                self._timed(plan, "fwd", plan._cur_stream, lambda: call("ym_conv_fwd_eval", *ev[1:], st))
                return
        ss, sq = self.ps[0], self.ps[1]
        conv = self.__dict__.get("_sc")
        if conv is None:
            conv = self._sc = (ctypes.byref(self.desc), self.x.ptr(), self.wf.data_ptr(), self.z.data_ptr(), None,
                               ss.data_ptr() if plan.training else None, sq.data_ptr() if plan.training else None)
        if plan.training and self._fused(plan):
            fold = self._fold(plan)
            self._timed(plan, "fwd", plan._cur_stream,
                        lambda: call("ym_conv_fwd_bn", conv[0], conv[1], conv[2], conv[3], conv[5], conv[6], fold, st))
            self._bn_fwd(plan, st, ss, sq, finalize=False)
            return
        self._timed(plan, "fwd", plan._cur_stream, lambda: call("ym_conv_fwd", *conv, st))
        self._bn_fwd(plan, st, ss, sq)

    def _bn_bwd(self, plan, st, dy):
        """BatchNorm (+ SiLU) backward: statistics pass over dy and z, finalize (dgamma, dbeta, apply
        coefficients), then dz = f(dy, z) written over z (+ the shortcut's gradient from the same dy
        read).  'bn' family: algorithmic bytes = dy + z read twice, dz written, partial rows, the
        shortcut gradient written (and read when it accumulates)."""
        bn = self.m.bn
        sc, sh, mu, rs = (self.bnv[i].data_ptr() for i in range(4))
        Gb = lib().ym_bn_bwd_blocks(self.M, self.co)
        r = self.res
        racc = r.grad_for_write(st) if r is not None else 0
        e = self.M * self.co * 2
        work = 5 * e + 16 * Gb * self.co + ((2 + racc) * e if r is not None else 0)

        fold = self.__dict__.get("_bwd_fold")
        if fold is None:
            fold = self._bwd_fold = bool(lib().ym_bn_bwd_fold_ok(self.M, self.co))
        fold = fold and os.environ.get("YM_BWD_FOLD", "1") == "1"

        def run():
            if fold:
                # small maps: statistics + finalize in one launch (the last workgroup of each 64-channel group folds)
                call("ym_bn_bwd_reduce_fold", dy, self.y.bs, self.y.ld, self.z.data_ptr(), self.M, self.co, self.HW,
                     sc, sh, mu, rs, self.act, self.ps[0].data_ptr(), self.ps[1].data_ptr(), _p(bn.weight),
                     plan.gptr(bn.weight), plan.gptr(bn.bias), 0, self.coef.data_ptr(), plan.bn_ws.data_ptr(), st)
            else:
                call("ym_bn_bwd_reduce", dy, self.y.bs, self.y.ld, self.z.data_ptr(), self.M, self.co, self.HW, sc,
                     sh, mu, rs, self.act, self.ps[0].data_ptr(), self.ps[1].data_ptr(), st)
                call("ym_bn_bwd_finalize", self.ps[0].data_ptr(), self.ps[1].data_ptr(), Gb, self.co, float(self.M),
                     _p(bn.weight), rs, plan.gptr(bn.weight), plan.gptr(bn.bias), 0, self.coef.data_ptr(),
                     plan.bn_ws.data_ptr(), st)
            if r is not None:
                call("ym_bn_bwd_apply_res", dy, self.y.bs, self.y.ld, self.z.data_ptr(), self.M, self.co, self.HW, sc,
                     sh, mu, rs, self.act, self.coef.data_ptr(), self.z.data_ptr(), r.gptr(), r.bs, r.ld, racc, st)
            else:
                call("ym_bn_bwd_apply", dy, self.y.bs, self.y.ld, self.z.data_ptr(), self.M, self.co, self.HW, sc, sh,
                     mu, rs, self.act, self.coef.data_ptr(), self.z.data_ptr(), st)
        self._timed(plan, "bn", plan._cur_stream, run, work)
        plan.note_grad_write(plan._cur_stream)          # dgamma / dbeta (finalize) are in the stream now
        if r is not None:
            r.mark()

    def backward(self, plan, st):
        dy = self.y.grad_for_read(st)
        self._bn_bwd(plan, st, dy)      # dz over z (z is needed by nobody after this op)
        dz = self.z
        # weight gradient: on the side stream, beside this layer's data gradient and the next BN backward
        ws = plan.wgrad_ws()
        sst = plan.side(st)
        self._timed(plan, "wgrad", plan.side_stream or plan._cur_stream, lambda: call(
            "ym_conv_wgrad", ctypes.byref(self.desc), dz.data_ptr(), self.x.ptr(), ws.data_ptr(), ws.numel() * 4,
            plan.gptr(self.m.conv.weight), 0, sst))
        plan.note_grad_write(plan.side_stream or plan._cur_stream)
        # data gradient
        if plan.needs_grad(self.x):
            acc = self.x.grad_for_write(st)
            self.desc.accumulate = acc
            self._timed(plan, "dgrad", plan._cur_stream, lambda: call(
                "ym_conv_dgrad", ctypes.byref(self.desc), dz.data_ptr(), self.wt.data_ptr(), self.x.gptr(), st))
            self.desc.accumulate = 0
            self.x.mark()


class StemConvBN(ConvBN):
    """model.0: Conv(ch -> c, 3x3 s2) on the fp32 NCHW image of ch = 1..4 planes (reference yaml backbone row 0;
    build_yolo11(ch=...), models/yolo11_model.py:23, 258)."""

    def rw(self, plan, phase):
        return ([], [_ka(self.y)]) if phase == "fwd" else ([_kg(self.y)], [_kg(self.y)])

    def __init__(self, plan, m, img_shape, y: View, s):
        w = m.conv.weight
        self.m, self.y, self.res, self.act, self.x = m, y, None, 1, None
        co, ci, k, _ = w.shape
        if not (1 <= ci <= 4 and k == 3):
            raise YolomiError(f"stem Conv({ci}, {co}, {k}): the stem kernels take 1..4 image planes and a 3x3 kernel")
        B, H, W = img_shape
        self.H, self.W, self.k, self.s, self.co, self.ci = H, W, k, s, co, ci
        oh, ow = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
        assert (oh, ow) == (y.H, y.W)
        self.M, self.HW, self.oh, self.ow = B * oh * ow, oh * ow, oh, ow
        self.z = torch.empty(self.M, co, dtype=BF16, device=plan.dev)
        self.G = 2048           # statistics rows = workgroups (2048 vs 1024: -22 us alone, +0.06-0.1 % step)
        self.ps = torch.empty(2, max(self.G, lib().ym_bn_bwd_blocks(self.M, co)), co, dtype=F32, device=plan.dev)
        self.bnv = torch.empty(4, co, dtype=F32, device=plan.dev)
        self.coef = torch.empty(3, co, dtype=F32, device=plan.dev)

    def _geo(self, plan):
        return (plan.B, self.H, self.W, self.oh, self.ow, self.co, self.s, 1)

    def forward(self, plan, st):
        y = self.y
        if (not plan.training and os.environ.get("YM_EVAL_FUSE", "1") != "0" and y.ptr() % 16 == 0 and y.ld % 8 == 0
                and y.bs % 8 == 0):
            # eval: conv + running-statistics BatchNorm + SiLU in one launch (ym_conv_first_fwd_eval)
            bn = self.m.bn
            (sc, sh, _, _), _, _, _ = self._static_args(plan)
            if not plan.eval_coeff_batched:
                call("ym_bn_eval_coeff", self.co, _p(bn.weight), _p(bn.bias), _p(bn.running_mean),
                     _p(bn.running_var), float(bn.eps), sc, sh, st)
            call("ym_conv_first_fwd_eval", plan.img.data_ptr(), _p(self.m.conv.weight), sc, sh, self.act, y.ptr(),
                 y.bs, y.ld, plan.B, self.H, self.W, self.oh, self.ow, self.co, self.s, 1, self.ci, st)
            return
        ss, sq = self.ps[0], self.ps[1]
        call("ym_conv_first_fwd", plan.img.data_ptr(), _p(self.m.conv.weight), self.z.data_ptr(), ss.data_ptr(),
             sq.data_ptr(), plan.B, self.H, self.W, self.oh, self.ow, self.co, self.s, 1, self.ci, self.G, st)
        self._bn_fwd(plan, st, ss, sq)

    def backward(self, plan, st):
        """Statistics pass + finalize as every Conv block, then the BatchNorm apply and the weight gradient in
        ONE pass over dy and the stored z (ym_stem_bwd_wgrad_stored: dz is never written and re-read; the
        kernel covers 16 / 32 / 64 channels of a 1-plane image — the n / s / m-l stems; other widths and multi-plane
        images: BN backward + a separate weight gradient over the written dz)."""
        dy = self.y.grad_for_read(st)
        if self.co not in (16, 32, 64) or self.ci != 1:
            self._bn_bwd(plan, st, dy)
            ws = plan.private_ws(self, lib().ym_conv_first_wgrad_workspace_size(self.co, self.ci))
            call("ym_conv_first_wgrad", self.z.data_ptr(), plan.img.data_ptr(), plan.gptr(self.m.conv.weight),
                 plan.B, self.H, self.W, self.oh, self.ow, self.co, self.s, 1, self.ci, ws.data_ptr(),
                 ws.numel() * 4, st)
            plan.note_grad_write(plan._cur_stream)      # conv.weight: after the BN event _bn_bwd noted
            return
        bn = self.m.bn
        sc, sh, mu, rs = (self.bnv[i].data_ptr() for i in range(4))
        Gb = lib().ym_bn_bwd_blocks(self.M, self.co)
        ws = plan.private_ws(self, lib().ym_stem_bwd_wgrad_workspace_size(self.co))
        e = self.M * self.co * 2

        def run():
            call("ym_bn_bwd_reduce", dy, self.y.bs, self.y.ld, self.z.data_ptr(), self.M, self.co, self.HW, sc, sh,
                 mu, rs, self.act, self.ps[0].data_ptr(), self.ps[1].data_ptr(), st)
            call("ym_bn_bwd_finalize", self.ps[0].data_ptr(), self.ps[1].data_ptr(), Gb, self.co, float(self.M),
                 _p(bn.weight), rs, plan.gptr(bn.weight), plan.gptr(bn.bias), 0, self.coef.data_ptr(),
                 plan.bn_ws.data_ptr(), st)
            call("ym_stem_bwd_wgrad_stored", dy, self.y.bs, self.y.ld, self.z.data_ptr(), plan.img.data_ptr(),
                 self.bnv.data_ptr(), self.coef.data_ptr(), plan.gptr(self.m.conv.weight), ws.data_ptr(),
                 ws.numel() * 4, *self._geo(plan), st)
        self._timed(plan, "bn", plan._cur_stream, run, 4 * e + 16 * Gb * self.co + 4 * plan.B * self.H * self.W)
        plan.note_grad_write(plan._cur_stream)          # dgamma / dbeta and conv.weight are in the stream now


class DWConvBN(ConvBN):
    """Attention.pe: depthwise 3x3 + BN (no act) on v, + the attention output as residual (:122, :134)."""

    def rw(self, plan, phase):
        if phase == "fwd":
            return [_ka(self.x), _ka(self.res)], [_ka(self.y)]
        return [_ka(self.x), _kg(self.y)], [_kg(self.y), _kg(self.res), _kg(self.x)]

    def __init__(self, plan, m, qkv: View, heads, kd, hd, y: View, res: View):
        self.m, self.x, self.y, self.res, self.act = m, qkv, y, res, 0
        C = heads * hd
        self.C, self.map = C, (hd, 2 * kd + hd, 2 * kd)     # gsz, gstride, goff
        self.k, self.co = 3, C
        self.M, self.HW = y.M, y.H * y.W
        self.z = torch.empty(self.M, C, dtype=BF16, device=plan.dev)
        self.G = 256
        self.ps = torch.empty(2, max(self.G, lib().ym_bn_bwd_blocks(self.M, C)), C, dtype=F32, device=plan.dev)
        self.bnv = torch.empty(4, C, dtype=F32, device=plan.dev)
        self.coef = torch.empty(3, C, dtype=F32, device=plan.dev)

    def forward(self, plan, st):
        gsz, gstr, goff = self.map
        y, r = self.y, self.res
        if (not plan.training and os.environ.get("YM_EVAL_FUSE", "1") != "0" and y.ptr() % 16 == 0 and y.ld % 8 == 0
                and y.bs % 8 == 0 and (r is None or (r.ptr() % 8 == 0 and r.ld % 4 == 0 and r.bs % 4 == 0))):
            # eval: depthwise conv + running-statistics BatchNorm + the residual in one launch (ym_dw3x3_fwd_eval)
            bn = self.m.bn
            (sc, sh, _, _), _, _, _ = self._static_args(plan)
            if not plan.eval_coeff_batched:
                call("ym_bn_eval_coeff", self.co, _p(bn.weight), _p(bn.bias), _p(bn.running_mean),
                     _p(bn.running_var), float(bn.eps), sc, sh, st)
            call("ym_dw3x3_fwd_eval", self.x.ptr(), self.x.bs, self.x.ld, gsz, gstr, goff, _p(self.m.conv.weight), sc,
                 sh, self.act, r.ptr() if r is not None else None, r.bs if r is not None else 0,
                 r.ld if r is not None else 0, y.ptr(), y.bs, y.ld, plan.B, y.H, y.W, self.C, st)
            return
        ss, sq = self.ps[0], self.ps[1]
        call("ym_dw3x3_fwd", self.x.ptr(), self.x.bs, self.x.ld, gsz, gstr, goff, _p(self.m.conv.weight),
             self.z.data_ptr(), ss.data_ptr(), sq.data_ptr(), plan.B, self.y.H, self.y.W, self.C, self.G, st)
        self._bn_fwd(plan, st, ss, sq)

    def backward(self, plan, st):
        dy = self.y.grad_for_read(st)
        self._bn_bwd(plan, st, dy)
        # dx into the v channels of dqkv (accumulate if the attention core wrote them already)
        hd, hs, goff = self.map
        heads = self.C // hd
        vch = np.zeros(self.x.act.C, bool)
        for h in range(heads):
            vch[self.x.c0 + h * hs + goff: self.x.c0 + h * hs + goff + hd] = True
        acc = int(self.x.act.written[vch].all())
        gsz, gstr, goff = self.map
        ws = plan.private_ws(self, lib().ym_dw3x3_bwd_workspace_size(self.C))
        call("ym_dw3x3_bwd", self.x.ptr(), self.x.bs, self.x.ld, gsz, gstr, goff, _p(self.m.conv.weight),
             self.z.data_ptr(), self.x.gptr(), self.x.bs, self.x.ld, plan.gptr(self.m.conv.weight), plan.B, self.y.H,
             self.y.W, self.C, acc, ws.data_ptr(), ws.numel() * 4, st)
        plan.note_grad_write(plan._cur_stream)          # conv.weight: after the BN event _bn_bwd noted
        self.x.act.written[vch] = True


class AttnCore:
    """softmax(q^T k * kd^-0.5) and v @ attn^T per head (Attention.forward :124-134)."""

    def rw(self, plan, phase):
        if phase == "fwd":
            return [_ka(self.qkv)], [_ka(self.out)]
        return [_ka(self.qkv), _ka(self.out), _kg(self.out)], [_kg(self.out), _kg(self.qkv)]

    def __init__(self, plan, qkv: View, heads, kd, hd, out: View):
        self.qkv, self.out, self.heads, self.kd, self.hd = qkv, out, heads, kd, hd
        self.N = qkv.H * qkv.W
        self.scale = kd ** -0.5
        self.lse = torch.empty(plan.B, heads, self.N, dtype=F32, device=plan.dev)
        ws = lib().ym_attn_workspace_size(plan.B, heads, self.N)
        self.ws = torch.empty(max(ws // 4, 1), dtype=F32, device=plan.dev)

    def forward(self, plan, st):
        call("ym_attn_fwd", self.qkv.ptr(), self.qkv.bs, self.qkv.ld, plan.B, self.heads, self.N, self.kd, self.hd,
             self.scale, self.out.ptr(), self.out.bs, self.out.ld, self.lse.data_ptr(), st)

    def backward(self, plan, st):
        dout = self.out.grad_for_read(st)
        q = self.qkv
        hs = 2 * self.kd + self.hd
        wr = q.act.written
        idx = lambda off, n: np.concatenate([np.arange(q.c0 + h * hs + off, q.c0 + h * hs + off + n)
                                             for h in range(self.heads)])
        iq, ik, iv = idx(0, self.kd), idx(self.kd, self.kd), idx(2 * self.kd, self.hd)
        acc = [int(wr[i].all()) for i in (iq, ik, iv)]
        call("ym_attn_bwd", q.ptr(), q.bs, q.ld, self.out.ptr(), self.out.bs, self.out.ld, dout, self.out.bs,
             self.out.ld, self.lse.data_ptr(), plan.B, self.heads, self.N, self.scale, self.ws.data_ptr(), q.gptr(),
             q.bs, q.ld, acc[0], acc[1], acc[2], st)
        for i in (iq, ik, iv):
            wr[i] = True


class SPPFPools:
    """SPPF's three chained nn.MaxPool2d(5, 1, 2) (yolo11_modules.py:100-104) on fp32 values.

    The chain is evaluated on the fp32 cv1 output (recomputed by its BN-apply) so the
    first-maximum routing of the backward sees the same ties as the fp32 reference
    (chained pools copy values, so exact ties are structural); the bf16 copies go to
    the concat slices for cv2."""

    def rw(self, plan, phase):
        sl = self.slices
        if phase == "fwd":
            return [_ka(sl[0])], [_ka(v) for v in sl[1:]]
        return [_kg(v) for v in sl[1:]], [_kg(v) for v in sl]

    def __init__(self, plan, cv1_op, slices):
        self.slices = slices                      # [s0 (cv1 out), s1, s2, s3]
        x = slices[0]
        self.M, self.C, self.H, self.W = x.M, x.c, x.H, x.W
        self.P = torch.empty(4, self.M, self.C, dtype=F32, device=plan.dev)   # fp32 chain values
        self.code = torch.empty(3, self.M, self.C, dtype=torch.uint8, device=plan.dev)   # window argmax
        self.G = torch.empty(2, self.M, self.C, dtype=F32, device=plan.dev)   # grad ping-pong
        cv1_op.out32 = self.P[0]

    def fused(self, plan):
        """The whole chain in one launch per direction (ym_sppf_fwd / _bwd, chain kept in LDS) when
        the map fits in LDS (ym_sppf_supported); otherwise one launch per pool."""
        sl = self.slices
        return (lib().ym_sppf_supported(self.H, self.W, self.C)
                and sl[1].bs == sl[2].bs == sl[3].bs and sl[1].ld == sl[2].ld == sl[3].ld)

    def forward(self, plan, st):
        if self.fused(plan):
            y1, y2, y3 = self.slices[1:]
            call("ym_sppf_fwd", self.P[0].data_ptr(), self.code.data_ptr(), y1.ptr(), y2.ptr(), y3.ptr(), y1.bs, y1.ld,
                 None, plan.B, self.H, self.W, self.C, st)
            return
        for j in range(3):
            y = self.slices[j + 1]
            call("ym_maxpool5_f32_fwd", self.P[j].data_ptr(), self.P[j + 1].data_ptr(), self.code[j].data_ptr(),
                 y.ptr(), y.bs, y.ld, plan.B, self.H, self.W, self.C, st)

    def backward(self, plan, st):
        if self.fused(plan):
            s0, s1, s2, s3 = self.slices
            g1, g2, g3 = s1.grad_for_read(st), s2.grad_for_read(st), s3.grad_for_read(st)
            acc = s0.grad_for_write(st)
            call("ym_sppf_bwd", self.code.data_ptr(), g1, g2, g3, s1.bs, s1.ld, s0.gptr(), s0.bs, s0.ld, acc, None,
                 plan.B, self.H, self.W, self.C, st)
            s0.mark()
            return
        HW = self.H * self.W
        cur = self.G[0]
        s3 = self.slices[3]
        call("ym_view_to_f32", s3.grad_for_read(st), s3.bs, s3.ld, cur.data_ptr(), self.M, self.C, HW, st)
        # pool j's output grad = its concat slice grad + the next pool's routed grad
        for j in (2, 1):
            nxt = self.G[(3 - j) % 2]
            sj = self.slices[j]
            call("ym_maxpool5_f32_bwd", self.code[j].data_ptr(), cur.data_ptr(), sj.grad_for_read(st), sj.bs, sj.ld,
                 nxt.data_ptr(), None, 0, 0, 0, plan.B, self.H, self.W, self.C, st)
            cur = nxt
        s0 = self.slices[0]
        acc = s0.grad_for_write(st)
        call("ym_maxpool5_f32_bwd", self.code[0].data_ptr(), cur.data_ptr(), None, 0, 0, None, s0.gptr(), s0.bs, s0.ld,
             acc, plan.B, self.H, self.W, self.C, st)
        s0.mark()


class Upsample2:
    """nn.Upsample(scale_factor=2, mode='nearest') (yaml head rows 11, 14)."""

    def rw(self, plan, phase):
        if phase == "fwd":
            return [_ka(self.x)], [_ka(self.y)]
        return [_kg(self.y)], [_kg(self.y), _kg(self.x)]

    def __init__(self, plan, x: View, y: View):
        self.x, self.y = x, y

    def forward(self, plan, st):
        x, y = self.x, self.y
        call("ym_upsample2_fwd", x.ptr(), x.bs, x.ld, y.ptr(), y.bs, y.ld, plan.B, x.H, x.W, x.c, st)

    def backward(self, plan, st):
        x, y = self.x, self.y
        dy = y.grad_for_read(st)
        acc = x.grad_for_write(st)
        call("ym_upsample2_bwd", dy, y.bs, y.ld, x.gptr(), x.bs, x.ld, plan.B, x.H, x.W, x.c, acc, st)
        x.mark()


class Copy:
    """Channel-slice copy for the two concatenations whose halves live in different buffers (PSA / C2PSA)."""

    def rw(self, plan, phase):
        if phase == "fwd":
            return [_ka(self.x)], [_ka(self.y)]
        return [_kg(self.y)], [_kg(self.y), _kg(self.x)]

    def __init__(self, plan, x: View, y: View):
        self.x, self.y = x, y

    def forward(self, plan, st):
        x, y = self.x, self.y
        call("ym_view_axpy", x.ptr(), x.bs, x.ld, y.ptr(), y.bs, y.ld, x.M, x.c, x.H * x.W, 0, 1, st)

    def backward(self, plan, st):
        x, y = self.x, self.y
        dy = y.grad_for_read(st)
        acc = x.grad_for_write(st)
        call("ym_view_axpy", dy, y.bs, y.ld, x.gptr(), x.bs, x.ld, x.M, x.c, x.H * x.W, acc, 0, st)
        x.mark()


class HeadLevel:
    """Detect level i: the two bias 1x1 convs (cv2[i][2] -> 64 box logits, cv3[i][2] -> nc cls logits)
    writing fp32 rows of the (B, A, 64+nc) head buffer (Detect.forward :237-246)."""

    def rw(self, plan, phase):
        if phase == "fwd":
            return [_ka(self.xb), _ka(self.xc)], [("head", self.a_off)]
        return [_ka(self.xb), _ka(self.xc), ("dhead", self.a_off)], [_kg(self.xb), _kg(self.xc)]

    def __init__(self, plan, box_conv, cls_conv, xb: View, xc: View, head, a_off):
        self.box, self.cls, self.xb, self.xc, self.head, self.a_off = box_conv, cls_conv, xb, xc, head, a_off
        B, A, no = head.shape
        self.nc = no - 64
        self.HW, self.M = xb.H * xb.W, B * xb.H * xb.W
        self.wb_f, self.wb_t = plan.weights.add(box_conv.weight, need_t=True)
        ncp = (self.nc + 7) // 8 * 8          # class gradient rows padded to 8 channels (ym_head_grad)
        self.wc_f, self.wc_t = plan.weights.add(cls_conv.weight, need_t=True, cout_t=ncp)
        self.dzb = torch.empty(self.M, 64, dtype=BF16, device=plan.dev)
        self.dzc = torch.empty(self.M, ncp, dtype=BF16, device=plan.dev)
        self.wsc = torch.empty(ncp, xc.c, dtype=F32, device=plan.dev)

        def desc(x, cout, y_bs, y_ld, out_f32):
            d = ConvDesc()
            d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout = B, x.H, x.W, x.c, x.H, x.W, cout
            d.k, d.stride, d.pad = 1, 1, 0
            d.x_bs, d.x_ld, d.y_bs, d.y_ld, d.out_f32 = x.bs, x.ld, y_bs, y_ld, out_f32
            return d
        self.fb = desc(xb, 64, A * no, no, 1)
        self.fc = desc(xc, self.nc, A * no, no, 1)
        self.bb = desc(xb, 64, self.HW * 64, 64, 0)
        self.bc = desc(xc, ncp, self.HW * ncp, ncp, 0)
        plan.need_wgrad_ws(self.bb)
        plan.need_wgrad_ws(self.bc)

    def forward(self, plan, st):
        base = self.head.data_ptr() + self.a_off * self.head.shape[2] * 4
        call("ym_conv_fwd", ctypes.byref(self.fb), self.xb.ptr(), self.wb_f.data_ptr(), base, _p(self.box.bias), None,
             None, st)
        call("ym_conv_fwd", ctypes.byref(self.fc), self.xc.ptr(), self.wc_f.data_ptr(), base + 64 * 4,
             _p(self.cls.bias), None, None, st)

    def backward(self, plan, st):
        B, A, no = self.head.shape
        ws = plan.private_ws(self, lib().ym_head_grad_workspace_size())
        call("ym_head_grad", plan.dhead.data_ptr(), A, self.a_off, self.HW, self.M, self.nc, self.dzb.data_ptr(),
             self.dzc.data_ptr(), plan.gptr(self.box.bias), plan.gptr(self.cls.bias), ws.data_ptr(), ws.numel() * 4,
             st)
        ws = plan.wgrad_ws()
        sst = plan.side(st)
        call("ym_conv_wgrad", ctypes.byref(self.bb), self.dzb.data_ptr(), self.xb.ptr(), ws.data_ptr(), ws.numel() * 4,
             plan.gptr(self.box.weight), 0, sst)
        call("ym_conv_wgrad", ctypes.byref(self.bc), self.dzc.data_ptr(), self.xc.ptr(), ws.data_ptr(), ws.numel() * 4,
             self.wsc.data_ptr(), 0, sst)
        g = plan.grad_view(self.cls.weight).view(self.nc, -1)
        with torch.cuda.stream(plan.side_stream or plan._cur_stream or torch.cuda.current_stream(plan.dev)):
            g.copy_(self.wsc[: self.nc])
        for d, dz, wt, x in ((self.bb, self.dzb, self.wb_t, self.xb), (self.bc, self.dzc, self.wc_t, self.xc)):
            acc = x.grad_for_write(st)
            d.accumulate = acc
            call("ym_conv_dgrad", ctypes.byref(d), dz.data_ptr(), wt.data_ptr(), x.gptr(), st)
            d.accumulate = 0
            x.mark()


def op_params(op):
    """Parameters whose gradients an op's backward finalises (in the flat gradient buffer)."""
    if isinstance(op, HeadLevel):
        mods = (op.box, op.cls)
    elif isinstance(op, ConvBN):
        mods = (op.m,)
    else:
        return []
    return [p for m in mods for p in m.parameters() if p.requires_grad]


# ----------------------------------------------------------------------------- plan
class Plan:
    def __init__(self, root, B, H, W, dev, training):
        self.root, self.B, self.dev, self.training = root, B, dev, training
        self.eval_coeff_batched = not training and dev.type == "cuda"   # one launch for every layer
        self.acts, self.ops = [], []
        self.weights = WeightStore(self)
        self.probe, self.probe_events = None, []   # bench: time one op's conv launch
        self.family_events = None  # bench: {'fwd'|'dgrad'|'wgrad': [(ev0, ev1, op)]} for every ConvBN launch
        self._bn_ws = []           # one BN-reduction workspace per scheduler stream (see bn_ws)
        self._cur = 0              # scheduler stream the current op runs on
        self.input = None          # View for block plans
        self.img = None            # fp32 image for the full model
        self.head = None           # (B, A, 64+nc) fp32 for the full model
        self.dhead = None
        self._scratch = []
        self.grad_hook = None      # called with each op's finished parameters during backward (DP buckets)
        self._writes = []          # (stream, event) after each parameter-gradient write of the current op
        self.on_op = None          # tools: called with (op index, op, phase) before each op runs (launch maps)
        self.side_stream = None    # weight-gradient stream (see side())
        self._cur_stream = None    # torch stream the current op is issued on (scheduler)
        # flat parameter-gradient buffer; each .grad is a view of it
        params = [p for p in root.parameters() if p.requires_grad]
        self.params = params
        sizes = [p.numel() for p in params]
        self.grad_flat = torch.zeros(max(sum(sizes), 1), dtype=F32, device=dev)
        self.grad_views, off = {}, 0
        for p, n in zip(params, sizes):
            self.grad_views[id(p)] = self.grad_flat[off:off + n].view(p.shape)
            off += n

    # --------------------------------------------------------------- side stream (weight gradients)
    # Weight gradients only read dz and the forward activation, and only write their own slice of
    # grad_flat, so they run on a second HIP stream: each conv's wgrad starts once its dz is ready
    # (an event on the main stream) and overlaps that layer's dgrad and the next ops' BN backward;
    # small late layers fill the chip together instead of each draining it.  The wgrads stay ordered
    # among themselves (they share the split-K workspace).  YM_SIDE_STREAM=0 runs them in line.
    def side(self, st):
        """Side-stream pointer for a launch that depends on everything issued so far on `st`."""
        s = self.side_stream
        if s is None:
            return st
        self._link(s, self._cur_stream or torch.cuda.current_stream(self.dev))
        return s.cuda_stream

    def _link(self, dst, src):
        """dst waits for everything issued so far on src, through ONE persistent event per source stream
        (re-recorded each time).  torch's wait_stream records a temporary event that is destroyed right
        after the wait; inside a HIP graph capture the runtime still refers to it at hipStreamEndCapture,
        which then crashed once the capture held several such joins (the 3-stream forward capture)."""
        evs = self.__dict__.setdefault("_link_events", {})
        ev = evs.get(src.cuda_stream)
        if ev is None:
            ev = evs[src.cuda_stream] = torch.cuda.Event()
        ev.record(src)
        dst.wait_event(ev)

    def note_grad_write(self, stream):
        """Under DP (a grad hook is set): record an event on `stream` right after a launch that wrote
        parameter gradients of the current op, so the bucket holding them waits for exactly that launch
        and not for the later, unrelated work of the same stream (the op's data gradient).  One
        persistent event per (op position, write), re-recorded every step."""
        if self.grad_hook is None or stream is None:
            return
        evs = self.__dict__.setdefault("_wevents", {})
        key = (self._op_pos, len(self._writes))
        ev = evs.get(key)
        if ev is None:
            ev = evs[key] = torch.cuda.Event()
        ev.record(stream)
        self._writes.append((stream, ev))

    def take_grad_writes(self, op):
        """The (stream, event) writes the op just noted; an op that noted none (the few that do not
        instrument their launches) is covered by its stream's and the side stream's tails."""
        w, self._writes = self._writes, []
        if not w and self.grad_hook is not None and self.dev.type == "cuda":
            for st in (self._cur_stream, self.side_stream):
                if st is not None:
                    self.note_grad_write(st)
            w, self._writes = self._writes, []
        return w

    def _begin_side(self):
        use = self.dev.type == "cuda" and os.environ.get("YM_SIDE_STREAM", "1") != "0"
        if use and self.side_stream is None:
            self.side_stream = torch.cuda.Stream(device=self.dev)
        elif not use:
            self.side_stream = None

    def _join_side(self):
        if self.side_stream is not None:
            self._link(torch.cuda.current_stream(self.dev), self.side_stream)

    def act(self, C, H, W, name=""):
        return View(Act(self, C, H, W, name=name))

    def private_ws(self, op, nbytes):
        """An op's own fp32 scratch (partial rows of its fixed-order reductions), allocated once."""
        ws = op.__dict__.get("_ws")
        if ws is None or ws.numel() * 4 < nbytes:
            ws = op.__dict__["_ws"] = torch.empty(max((nbytes + 3) // 4, 1), dtype=F32, device=self.dev)
        return ws

    def need_wgrad_ws(self, desc):
        """Size the shared split-K workspace of ym_conv_wgrad (ops run in order on one stream)."""
        self._wg_bytes = max(getattr(self, "_wg_bytes", 0), int(lib().ym_conv_wgrad_workspace_size(ctypes.byref(desc))))

    def _alloc_bn_ws(self, K):
        """Allocate the BN scratch of K scheduler streams, zeroed once (the one-launch finalize's
        ticket counters live at offset 0 and re-arm themselves).  Runs on the caller's stream
        before the other streams fork from it, so the zero fill is ordered before every op that
        takes a ticket."""
        while len(self._bn_ws) < K:
            self._bn_ws.append(torch.zeros((lib().ym_bn_workspace_size(2048) + 3) // 4, dtype=F32, device=self.dev))

    @property
    def bn_ws(self):
        """BatchNorm reduction scratch of the stream the current op runs on (ops on different
        streams run concurrently, so each stream has its own)."""
        if len(self._bn_ws) <= self._cur:
            raise YolomiError("BN workspace of a scheduler stream used before _run allocated it")
        return self._bn_ws[self._cur]

    def wgrad_ws(self):
        """Split-K scratch of ym_conv_wgrad: one for the side stream (wgrads run there in order), or
        one per scheduler stream when they run in line."""
        key = -1 if self.side_stream is not None else self._cur
        wss = self.__dict__.setdefault("_wg_ws", {})
        if key not in wss:
            wss[key] = torch.empty(max(self._wg_bytes // 4, 1), dtype=F32, device=self.dev)
        return wss[key]

    def grad_view(self, p):
        return self.grad_views[id(p)]

    def gptr(self, p):
        if p is None or not p.requires_grad:
            return None
        return self.grad_views[id(p)].data_ptr()

    def needs_grad(self, v: View):
        return v.act is not None and (v.act is not getattr(self.input, "act", None) or self.input_requires_grad)

    # --------------------------------------------------------------- stream scheduler
    # The op list is a DAG over buffer ranges (each op declares what it reads and writes, `rw`):
    # independent branches — the six Detect-head chains, C3k's two 1x1 branches, the concat
    # producers of C2f — run on different HIP streams, so the small 20x20 / 40x40 layers and the
    # latency-bound BatchNorm reductions of one chain overlap another chain's kernels.  The
    # schedule (stream per op + the events it waits for) is computed once per plan and phase:
    # an op follows the stream of its latest dependency while that stream's tail is that
    # dependency, otherwise it takes a stream whose tail it depends on, or the least recently used
    # one.  YM_STREAMS sets the stream count (1 = everything in order on the caller's stream).
    def _nstreams(self):
        if self.dev.type != "cuda":
            return 1
        if not self.training and self._graph_ok() and "YM_STREAMS" not in os.environ:
            # an eval forward replayed as a HIP graph: ONE stream (bs1 s@640 1.50 ms per batch vs 1.83 with the three
            # streams captured, same box, profiles/r05/eval_graph_streams.txt: the replayed cross-stream edges cost
            # more than the overlap they allow at these sizes)
            return 1
        k = max(1, int(os.environ.get("YM_STREAMS", "3")))
        return k

    def _schedule(self, ops, phase, K):
        key = (phase, K, len(ops))
        cache = self.__dict__.setdefault("_sched", {})
        if key in cache:
            return cache[key]
        rws = [op.rw(self, phase) for op in ops]
        writes, reads, deps = [], [], []
        for i, (R, W) in enumerate(rws):
            d = set()
            for k in R:
                d.update(j for k2, j in writes if _overlap(k, k2))
            for k in W:
                d.update(j for k2, j in writes if _overlap(k, k2))
                d.update(j for k2, j in reads if _overlap(k, k2))
            deps.append(d)
            writes.extend((k, i) for k in W)
            reads.extend((k, i) for k in R)
        stream_of, tail, plan = [0] * len(ops), [-1] * K, []
        need_ev = set()
        for i, d in enumerate(deps):
            s = 0
            if d:
                j = max(d)
                s = stream_of[j]
                if tail[s] != j:
                    cands = [t for t in range(K) if tail[t] in d]
                    s = max(cands, key=lambda t: tail[t]) if cands else min(range(K), key=lambda t: tail[t])
            elif i > 0:
                s = min(range(K), key=lambda t: tail[t])
            waits = {}
            for j in d:
                if stream_of[j] != s:
                    waits[stream_of[j]] = max(waits.get(stream_of[j], -1), j)
            stream_of[i] = s
            tail[s] = i
            need_ev.update(waits.values())
            plan.append((s, sorted(waits.values())))
        cache[key] = (plan, need_ev)
        return cache[key]

    def _streams(self, K):
        ss = self.__dict__.setdefault("_dag_streams", [])
        while len(ss) < K - 1:
            ss.append(torch.cuda.Stream(device=self.dev))
        return [torch.cuda.current_stream(self.dev)] + ss[:K - 1]

    def comm_streams(self):
        """Every stream a backward writes gradients from (the DP buckets join them before a collective)."""
        out = list(self.__dict__.get("_active_streams", []))
        if self.side_stream is not None:
            out.append(self.side_stream)
        return out

    def _run(self, ops, phase, after=None):
        K = self._nstreams()
        if phase == "fwd" and os.environ.get("YM_FWD_STREAMS"):
            K = max(1, int(os.environ["YM_FWD_STREAMS"]))      # A/B runs: the forward's stream count alone
        self._alloc_bn_ws(K)
        if K == 1:
            st = stream_ptr(self.dev)
            self._cur = 0
            self._active_streams = [torch.cuda.current_stream(self.dev)]
            self._cur_stream = self._active_streams[0]
            for i, op in enumerate(ops):
                self._op_pos = i
                if self.on_op is not None:
                    self.on_op(i, op, phase)
                getattr(op, phase == "fwd" and "forward" or "backward")(self, st)
                if after is not None:
                    after(op)
            return
        sched, need_ev = self._schedule(ops, phase, K)
        streams = self._streams(K)
        self._active_streams = streams
        evs = self.__dict__.setdefault("_events", {}).setdefault(phase, {})
        main = streams[0]
        for s in streams[1:]:
            self._link(s, main)
        ptrs = [s.cuda_stream for s in streams]
        fwd = phase == "fwd"
        # HIP graph capture (ROCm 7.2 runtime) segfaults in hipStreamEndCapture once two non-origin streams
        # have waited on each other's events (tools/hip_graph_repro.py `cycle`: s2 waits on s1, later s1 on
        # s2 — four torch calls, no yolomi code).  While capturing, such a wait is relayed through the origin
        # stream (main waits on the producer's event, the consumer on main's), which captures and replays
        # correctly (`sched46_relay`); eager runs keep the direct wait.
        relay = torch.cuda.is_current_stream_capturing()
        # ops launch on explicit stream handles (no torch stream context per op: it is host time the
        # GPU waits for); the few torch-side launches (side-stream joins, probe events) use _cur_stream
        for i, op in enumerate(ops):
            k, waits = sched[i]
            s = streams[k]
            for j in waits:
                if relay and k != 0 and sched[j][0] != 0:
                    main.wait_event(evs[j])
                    self._link(s, main)
                else:
                    s.wait_event(evs[j])
            self._cur, self._cur_stream = k, s
            self._op_pos = i
            if self.on_op is not None:
                self.on_op(i, op, phase)
            if fwd:
                op.forward(self, ptrs[k])
            else:
                op.backward(self, ptrs[k])
            if after is not None:
                after(op)
            if i in need_ev:
                ev = evs.get(i)
                if ev is None:
                    ev = evs[i] = torch.cuda.Event()
                ev.record(s)
        for s in streams[1:]:
            self._link(main, s)
        self._cur, self._cur_stream = 0, None

    # --------------------------------------------------------------- HIP graphs
    # After one eager run (which allocates every workspace, stream and event), the whole forward
    # and the whole backward of a model plan are captured once each as HIP graphs (all streams,
    # events and kernels) and replayed: the per-step host work drops from ~900 ctypes launches to
    # two graph launches, so the GPU no longer waits on Python between kernels.  The captured
    # launches point at fixed buffers: the input image and the head gradient are copied into the
    # plan's own static tensors when the caller's differ.  Not used while the bench probe times a
    # kernel with events, or for block plans.  Data parallelism in graph mode all-reduces the flat
    # gradient once after the backward (yolomi/dist.py).  Training: opt-in (YM_GRAPH=1): the step is
    # GPU-bound (host enqueue ~8 ms of a ~20 ms step), so replay has no host time to win back (DESIGN.md
    # §10).  Eval: on by default (YM_EVAL_GRAPH=0 opts out), captured on ONE stream (_nstreams): a bs-1
    # eval forward is ~100 launches of a few us each whose Python enqueue leaves the GPU idle between
    # them (bs1 s@640: 1.50 ms per batch replayed vs 1.83 eager on three streams, same box,
    # profiles/r05/eval_graph_streams.txt).  A captured graph holds raw pointers, so every
    # call compares the pointers of the model's parameters and buffers with the captured ones
    # (_graph_key) and re-captures after an eager run when one was replaced.
    def _graph_ok(self):
        if not (self.dev.type == "cuda" and getattr(self, "is_model", False) and self.probe is None
                and self.family_events is None):
            return False
        if self.training:
            return os.environ.get("YM_GRAPH", "0") == "1"
        return os.environ.get("YM_EVAL_GRAPH", "1") == "1"

    def _graph_key(self):
        """Data pointers of every parameter and buffer of the model, looked up in the modules' live
        dictionaries (a replaced Parameter / buffer is seen)."""
        pairs = self.__dict__.get("_gk_pairs")
        if pairs is None:
            pairs = self._gk_pairs = []
            for mod in self.root.modules():
                pairs += [(mod._parameters, n) for n in mod._parameters]
                pairs += [(mod._buffers, n) for n in mod._buffers]
        # + the library's policy generation: a graph captured under one kernel-selection policy is not replayed under
        # another (yolomi_experimental.h)
        return tuple(t.data_ptr() if t is not None else 0 for t in (d.get(n) for d, n in pairs)) + (
            lib().ym_policy_generation(),)

    @property
    def graph_active(self):
        return self._graph_ok()

    def _replay(self, phase, body, static_in):
        """Eager on the first call of a phase, capture on the second, replay afterwards.
        static_in: list of (attribute name, tensor) inputs the captured kernels read by address.
        A capture only follows an eager run over the same parameter / buffer pointers: the eager run
        rebuilds the pointer tables (weight preparation, eval coefficients) and uploads them, which a
        capture must not do.  A replaced parameter or buffer drops the graph (eager, then capture again)."""
        graphs = self.__dict__.setdefault("_graphs", {})
        eager_keys = self.__dict__.setdefault("_eager_keys", {})
        if not self._graph_ok():
            body()
            return
        key = self._graph_key()
        ent = graphs.get(phase)
        if ent is not None and ent[2] != key:
            del graphs[phase]
            ent = None
        if ent is None and eager_keys.get(phase) != key:
            eager_keys[phase] = key
            body()
            return
        if ent is None:
            statics = {}
            for name, t in static_in:
                statics[name] = torch.empty_like(t)
                statics[name].copy_(t)
                setattr(self, name, statics[name])
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(self.dev)
            # thread_local: only THIS thread's HIP calls are checked against the capture — the DataLoader's
            # pin-memory thread (validate(): the capture is the second val batch) and the process group's
            # watchdog keep running during it instead of erroring or invalidating the capture
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                body()
            graphs[phase] = ent = (g, statics, key)
        g, statics, _ = ent
        for name, t in static_in:
            st_t = statics[name]
            if t.data_ptr() != st_t.data_ptr():
                st_t.copy_(t)
            setattr(self, name, st_t)
        g.replay()

    # --------------------------------------------------------------- run
    def _eval_coeffs(self, st):
        """Eval: every BatchNorm layer's scale / shift from its running statistics in ONE launch
        (ym_bn_eval_coeff_batch over a pointer table built once per plan; the parameters and buffers
        are read at launch time, so later weight / statistics updates are picked up)."""
        ents = [op for op in self.ops if hasattr(op, "bnv") and hasattr(op, "m")]
        # keyed on EVERY pointer the table holds: a parameter or buffer replaced by a new tensor
        # (load_state_dict(assign=True), bn.running_var = ...) rebuilds it instead of leaving a dangling one
        key = tuple((_p(op.m.bn.weight), _p(op.m.bn.bias), _p(op.m.bn.running_mean), _p(op.m.bn.running_var),
                     op.bnv.data_ptr()) for op in ents)
        if getattr(self, "_eval_key", None) != key:
            arr = (BnEvalEntry * len(ents))()
            for e, op in zip(arr, ents):
                bn = op.m.bn
                e.gamma, e.beta = _p(bn.weight), _p(bn.bias)
                e.running_mean, e.running_var = _p(bn.running_mean), _p(bn.running_var)
                e.scale, e.shift = op.bnv[0].data_ptr(), op.bnv[1].data_ptr()
                e.c, e.eps = op.bnv.shape[1], float(bn.eps)
            self._eval_table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.dev)
            self._eval_n = len(ents)
            self._eval_key = key
        call("ym_bn_eval_coeff_batch", self._eval_table.data_ptr(), self._eval_n, st)

    def forward(self):
        def body():
            st = stream_ptr(self.dev)
            self.weights.refresh(st)
            if self.eval_coeff_batched:
                self._eval_coeffs(st)
            self._run(self.ops, "fwd")
        self._replay("fwd", body, [("img", self.img)] if self.img is not None else [])

    def backward(self):
        # gradient accumulation without zero_grad(): the parameters' .grad still alias this plan's flat
        # buffer (install_grads) and hold the previous backward's sum, which the zero fill of the backward
        # would drop — keep it and add it back after this backward (single-process; under DP the buffer is
        # on the wire during the backward, and the reference's loop zeroes its gradients every step).
        # Decided and done eagerly, OUTSIDE the body a HIP graph captures and replays (YM_GRAPH=1): a
        # captured decision would replay a stale keep buffer, or none, on every later step.
        keep = self._accumulation_keep()
        self._replay("bwd", lambda: self._backward_ops(self.ops),
                     [("dhead", self.dhead)] if self.dhead is not None else [])
        if keep is not None:
            self.grad_flat.add_(keep)

    def _accumulation_keep(self):
        if self.grad_hook is None and self.params:
            p0 = self.params[0]
            if p0.grad is not None and p0.grad.data_ptr() == self.grad_views[id(p0)].data_ptr():
                return self.grad_flat.clone()
        return None

    def _backward_ops(self, ops):
        for a in self.acts:
            a.written[:] = False
        self.grad_flat.zero_()
        for t in self._scratch:
            t.zero_()
        hook = None if self._graph_ok() else self.grad_hook
        self._begin_side()
        self._writes = []
        self._run(list(reversed(ops)), "bwd",
                  (lambda op: hook(op_params(op), self.take_grad_writes(op))) if hook is not None else None)
        self._join_side()

    # --------------------------------------------------------------- forwards in flight
    # A plan owns ONE set of activation buffers.  While a training forward's autograd graph is alive
    # and its backward has not run, the plan is "pending" (a weak reference to the graph node); the
    # next forward of the same shape then takes another plan of the model's pool for that shape (its
    # own activation set, the same parameters), as the reference's autograd keeps one set of saved
    # tensors per forward (train_yolo11_cuda.py:51-57).  A plan is reused once its backward has run or
    # its graph has been freed.  The generation check stays as a guard: a backward whose plan has since
    # run another forward raises instead of returning wrong gradients, and so does a second backward
    # through one forward (the backward overwrites z with dz in place).
    def new_generation(self):
        self.gen = getattr(self, "gen", 0) + 1
        return self.gen

    def check_generation(self, gen):
        if gen != getattr(self, "gen", 0):
            raise YolomiError("backward of a forward whose activations a newer forward of the same input shape has "
                              "overwritten: run backward (or detach the outputs) before the next forward")

    def set_pending(self, ctx):
        self._pending = weakref.ref(ctx) if ctx is not None else None

    @property
    def pending(self):
        r = self.__dict__.get("_pending")
        return r is not None and r() is not None

    def install_grads(self):
        """Expose the flat buffer as parameter .grad (accumulating if a grad already exists)."""
        for p in self.params:
            g = self.grad_views[id(p)]
            if p.grad is None:
                p.grad = g
            elif p.grad.data_ptr() != g.data_ptr():
                p.grad.add_(g)


# ----------------------------------------------------------------------------- lowering
def _conv(plan, m, x: View, out: View | None = None, res=None, act=None):
    k, s = m.conv.kernel_size[0], m.conv.stride[0]
    co = m.conv.out_channels
    H, W = (x.H + 2 * (k // 2) - k) // s + 1, (x.W + 2 * (k // 2) - k) // s + 1
    y = out if out is not None else plan.act(co, H, W)
    if act is None:
        act = not isinstance(m.act, torch.nn.Identity)
    plan.ops.append(ConvBN(plan, m, x, y, s, act, res))
    return y


def _bottleneck(plan, m, x: View, out=None):
    t = _conv(plan, m.cv1, x)
    return _conv(plan, m.cv2, t, out, res=x if m.add else None)


def _c3k(plan, m, x: View, out=None):
    c_ = m.cv1.conv.out_channels
    cat = plan.act(2 * c_, x.H, x.W)
    a = _conv(plan, m.cv1, x)
    blocks = list(m.m)
    for j, b in enumerate(blocks):
        a = _bottleneck(plan, b, a, cat.sub(0, c_) if j == len(blocks) - 1 else None)
    _conv(plan, m.cv2, x, cat.sub(c_, c_))
    return _conv(plan, m.cv3, cat, out)


def _c2f(plan, m, x: View, out=None):
    c, n = m.c, len(m.m)
    cat = plan.act((2 + n) * c, x.H, x.W)
    _conv(plan, m.cv1, x, cat.sub(0, 2 * c))
    prev = cat.sub(c, c)
    for j, b in enumerate(m.m):
        dst = cat.sub((2 + j) * c, c)
        if type(b).__name__ == "C3k":
            prev = _c3k(plan, b, prev, dst)
        else:
            prev = _bottleneck(plan, b, prev, dst)
    return _conv(plan, m.cv2, cat, out)


def _sppf(plan, m, x: View, out=None):
    c_ = m.cv1.conv.out_channels
    cat = plan.act(4 * c_, x.H, x.W)
    _conv(plan, m.cv1, x, cat.sub(0, c_))
    plan.ops.append(SPPFPools(plan, plan.ops[-1], [cat.sub(j * c_, c_) for j in range(4)]))
    return _conv(plan, m.cv2, cat, out)


def _attention(plan, m, x: View, out: View, res: View):
    heads, kd, hd = m.num_heads, m.key_dim, m.head_dim
    qkv = _conv(plan, m.qkv, x, act=False)
    o = plan.act(heads * hd, x.H, x.W)
    plan.ops.append(AttnCore(plan, qkv, heads, kd, hd, o))
    s = plan.act(heads * hd, x.H, x.W)
    plan.ops.append(DWConvBN(plan, m.pe, qkv, heads, kd, hd, s, o))
    return _conv(plan, m.proj, s, out, res=res, act=False)


def _psa(plan, m, x: View, out=None):
    c = m.c
    cat = plan.act(2 * c, x.H, x.W)
    # eval plans: cv1 writes [a | b] straight into the concat and b3 overwrites b there (b is dead once the attention's
    # qkv conv and its residual have read it; the scheduler orders that write after those reads) — no copy of a.
    # Training keeps b: the backward reads it (the qkv conv's weight gradient)
    y = _conv(plan, m.cv1, x, None if plan.training else cat)      # [a | b]
    a, b = y.sub(0, c), y.sub(c, c)
    b2 = plan.act(c, x.H, x.W)
    _attention(plan, m.attn, b, b2, res=b)         # b2 = b + attn(b)
    f1 = _conv(plan, m.ffn[0], b2)
    _conv(plan, m.ffn[1], f1, cat.sub(c, c), res=b2, act=False)   # b3 = b2 + ffn(b2)
    if plan.training:
        plan.ops.append(Copy(plan, a, cat.sub(0, c)))
    return _conv(plan, m.cv2, cat, out)


def _c2psa(plan, m, x: View, out=None):
    c = m.c
    cat = plan.act(2 * c, x.H, x.W)
    # eval plans: as in _psa, cv1's [a | b] lands in the concat and the last PSA block's output overwrites b there
    y = _conv(plan, m.cv1, x, None if plan.training else cat)
    a, b = y.sub(0, c), y.sub(c, c)
    blocks = list(m.m)
    for j, blk in enumerate(blocks):
        b = _psa(plan, blk, b, cat.sub(c, c) if j == len(blocks) - 1 else None)
    if plan.training:
        plan.ops.append(Copy(plan, a, cat.sub(0, c)))
    return _conv(plan, m.cv2, cat, out)


def _detect(plan, m, xs, head):
    a_off = 0
    for i, x in enumerate(xs):
        b = _conv(plan, m.cv2[i][1], _conv(plan, m.cv2[i][0], x))
        c = _conv(plan, m.cv3[i][1], _conv(plan, m.cv3[i][0], x))
        plan.ops.append(HeadLevel(plan, m.cv2[i][2], m.cv3[i][2], b, c, head, a_off))
        a_off += x.H * x.W


def _attention_block(plan, m, x: View, out=None):
    """Attention.forward on its own (yolo11_modules.py:124-136): proj(attn(x) + pe(v)), no residual."""
    return _attention(plan, m, x, out, res=None)


LOWER = {"Conv": _conv, "Bottleneck": _bottleneck, "C3k": _c3k, "C2f": _c2f, "C3k2": _c2f, "SPPF": _sppf,
         "C2PSA": _c2psa, "PSA": _psa, "Attention": _attention_block}


def lower_block(plan, m, x: View):
    t = type(m).__name__
    if t not in LOWER:
        raise YolomiError(f"no MI355X lowering for module type {t}")
    return LOWER[t](plan, m, x)


def lower_model(plan, model, img_shape):
    """YOLOv11._forward_once (yolo11_model.py:60-71) over the layer list with concat-slice planning."""
    layers = list(model.model)
    B, H, W = img_shape
    # output channels / spatial size of every layer
    shapes = []
    for i, L in enumerate(layers):
        t = type(L).__name__
        f = L.f
        src = (i - 1 if f == -1 else f) if isinstance(f, int) else None
        inp = (1, H, W) if (isinstance(f, int) and src < 0) else (shapes[src] if src is not None else None)
        if t == "Conv":
            k, s = L.conv.kernel_size[0], L.conv.stride[0]
            shapes.append((L.conv.out_channels, (inp[1] + 2 * (k // 2) - k) // s + 1,
                           (inp[2] + 2 * (k // 2) - k) // s + 1))
        elif t in ("C3k2", "C2f", "SPPF", "C2PSA"):
            shapes.append((L.cv2.conv.out_channels, inp[1], inp[2]))
        elif t == "Upsample":
            shapes.append((inp[0], inp[1] * 2, inp[2] * 2))
        elif t == "Concat":
            srcs = [shapes[i - 1 if j == -1 else j] for j in f]
            assert all(s_[1:] == srcs[0][1:] for s_ in srcs), f"concat {i}: spatial mismatch {srcs}"
            shapes.append((sum(s_[0] for s_ in srcs), srcs[0][1], srcs[0][2]))
        elif t == "Detect":
            shapes.append(None)
        else:
            raise YolomiError(f"no MI355X lowering for layer type {t}")
    # concat buffers: producers write into their slice
    dest = {}
    for i, L in enumerate(layers):
        if type(L).__name__ == "Concat":
            C, hh, ww = shapes[i]
            buf = plan.act(C, hh, ww, name=f"cat{i}")
            c0 = 0
            for j in L.f:
                src = i - 1 if j == -1 else j
                cj = shapes[src][0]
                assert src not in dest, "a layer feeding two concats is not supported"
                dest[src] = buf.sub(c0, cj)
                c0 += cj
            dest[i] = buf
    outs = []
    x = None
    for i, L in enumerate(layers):
        t = type(L).__name__
        f = L.f
        if f != -1:
            xin = outs[f] if isinstance(f, int) else [x if j == -1 else outs[j] for j in f]
        else:
            xin = x
        if t == "Conv":
            if i == 0:
                y = dest.get(i) or plan.act(*shapes[i])
                plan.ops.append(StemConvBN(plan, L, img_shape, y, L.conv.stride[0]))
                x = y
            else:
                x = _conv(plan, L, xin, dest.get(i))
        elif t in ("C3k2", "C2f"):
            x = _c2f(plan, L, xin, dest.get(i))
        elif t == "SPPF":
            x = _sppf(plan, L, xin, dest.get(i))
        elif t == "C2PSA":
            x = _c2psa(plan, L, xin, dest.get(i))
        elif t == "Upsample":
            y = dest.get(i) or plan.act(*shapes[i])
            plan.ops.append(Upsample2(plan, xin, y))
            x = y
        elif t == "Concat":
            x = dest[i]
        elif t == "Detect":
            nc = L.nc
            A = sum(v.H * v.W for v in xin)
            plan.head = torch.empty(B, A, 64 + nc, dtype=F32, device=plan.dev)
            plan.dhead = torch.empty_like(plan.head)
            _detect(plan, L, xin, plan.head)
            plan.level_hw = [(v.H, v.W) for v in xin]
            x = None
        outs.append(x)
    plan.layer_outs = outs
    return plan


# ----------------------------------------------------------------------------- autograd glue
class _ModelFn(torch.autograd.Function):
    """Whole-model forward/backward as one node; parameter grads are written into the plan's flat buffer."""

    @staticmethod
    def forward(ctx, img, anchor, plan):
        plan.img = img.contiguous()
        plan.forward()
        ctx.plan, ctx.gen = plan, plan.new_generation()
        plan.set_pending(ctx)
        return plan.head.detach()

    @staticmethod
    def backward(ctx, dhead):
        plan = ctx.plan
        plan.check_generation(ctx.gen)
        if getattr(ctx, "done", False):
            raise YolomiError("a second backward through one forward (retain_graph=True): the first backward "
                              "consumed the forward's activations in place; run the forward again")
        ctx.done = True
        plan.set_pending(None)
        plan.dhead = dhead.contiguous()
        plan.backward()
        plan.install_grads()
        return None, None, None


class _BlockFn(torch.autograd.Function):
    """A single building block on NCHW fp32 tensors (per-block parity / module-level API)."""

    @staticmethod
    def forward(ctx, x, anchor, plan):
        if plan.stem:
            plan.img = x.float().contiguous()
        else:
            plan.input.act.t.copy_(x.permute(0, 2, 3, 1))
        plan.forward()
        ctx.plan, ctx.gen = plan, plan.new_generation()
        out = plan.output.act.t[..., plan.output.c0:plan.output.c0 + plan.output.c]
        return out.permute(0, 3, 1, 2).float().contiguous()

    @staticmethod
    def backward(ctx, dy):
        plan = ctx.plan
        plan.check_generation(ctx.gen)
        o = plan.output
        g = o.act.grad()
        g[..., o.c0:o.c0 + o.c].copy_(dy.permute(0, 2, 3, 1))
        plan.backward_from_output()
        plan.install_grads()
        dx = plan.input.act.grad().permute(0, 3, 1, 2).float() if plan.input_requires_grad else None
        return dx, None, None


def run_block(module, x: torch.Tensor):
    """Execute one building block on the GPU through the plan (training or eval per module.training)."""
    if not x.is_cuda:
        raise YolomiError("yolomi kernels run on the MI355X only (got a CPU tensor)")
    B, C, H, W = x.shape
    key = ("block", B, H, W, module.training, x.requires_grad)
    cache = module.__dict__.setdefault("_ym_plans", {})
    plan = cache.get(key)
    if plan is None:
        plan = Plan(module, B, H, W, x.device, module.training)
        if type(module).__name__ == "Conv" and module.conv.in_channels <= 4 and module.conv.kernel_size[0] == 3:
            # stem conv reads the fp32 image directly (no input gradient)
            plan.stem = True
            plan.input = None
            plan.input_requires_grad = False
            k, s = module.conv.kernel_size[0], module.conv.stride[0]
            plan.output = plan.act(module.conv.out_channels, (H + 2 * (k // 2) - k) // s + 1,
                                   (W + 2 * (k // 2) - k) // s + 1)
            plan.ops.append(StemConvBN(plan, module, (B, H, W), plan.output, s))
        else:
            plan.stem = False
            plan.input = plan.act(C, H, W, name="input")
            plan.input_requires_grad = x.requires_grad
            plan.output = lower_block(plan, module, plan.input)

        def backward_from_output():
            for a in plan.acts:
                a.written[:] = False
            plan.grad_flat.zero_()
            for t in plan._scratch:
                t.zero_()
            plan.output.mark()
            plan._begin_side()
            plan._run(list(reversed(plan.ops)), "bwd")
            plan._join_side()
        plan.backward_from_output = backward_from_output
        cache[key] = plan
    anchor = module.__dict__.setdefault("_ym_anchor", torch.zeros(1, requires_grad=True))
    return _BlockFn.apply(x, anchor, plan)


class _DetectFn(torch.autograd.Function):
    """Detect on its own: three NCHW fp32 level maps -> the (B, A, 64+nc) fp32 head buffer."""

    @staticmethod
    def forward(ctx, anchor, plan, *xs):
        for v, x in zip(plan.inputs, xs):
            v.act.t.copy_(x.permute(0, 2, 3, 1))
        plan.forward()
        ctx.plan, ctx.gen = plan, plan.new_generation()
        ctx.needs = [x.requires_grad for x in xs]
        return plan.head.clone()

    @staticmethod
    def backward(ctx, dhead):
        plan = ctx.plan
        plan.check_generation(ctx.gen)
        plan.dhead = dhead.contiguous()
        plan.backward_from_head()
        plan.install_grads()
        dxs = [v.act.grad().permute(0, 3, 1, 2).float() if need else None for v, need in zip(plan.inputs, ctx.needs)]
        return (None, None, *dxs)


def run_detect(det, xs):
    """Detect.forward on standalone level maps (yolo11_modules.py:237-266): the head's six conv
    chains and bias convs as one plan; returns (head (B, A, 64+nc) fp32, plan)."""
    xs = list(xs)
    if not xs or not all(x.is_cuda for x in xs):
        raise YolomiError("yolomi kernels run on the MI355X only (got a CPU tensor)")
    if len(xs) != det.nl:
        raise YolomiError(f"Detect expects {det.nl} level maps, got {len(xs)}")
    B = xs[0].shape[0]
    key = ("detect", tuple(tuple(x.shape) for x in xs), det.training, tuple(x.requires_grad for x in xs))
    cache = det.__dict__.setdefault("_ym_plans", {})
    plan = cache.get(key)
    if plan is None:
        plan = Plan(det, B, xs[0].shape[2], xs[0].shape[3], xs[0].device, det.training)
        plan.inputs = [plan.act(x.shape[1], x.shape[2], x.shape[3], name=f"level{i}") for i, x in enumerate(xs)]
        plan.input = None
        plan.input_requires_grad = any(x.requires_grad for x in xs)
        A = sum(x.shape[2] * x.shape[3] for x in xs)
        plan.head = torch.empty(B, A, det.no, dtype=F32, device=plan.dev)
        plan.dhead = torch.empty_like(plan.head)
        _detect(plan, det, plan.inputs, plan.head)
        plan.level_hw = [(x.shape[2], x.shape[3]) for x in xs]

        def backward_from_head():
            keep = plan._accumulation_keep()
            plan._backward_ops(plan.ops)
            if keep is not None:
                plan.grad_flat.add_(keep)
        plan.backward_from_head = backward_from_head
        cache[key] = plan
    # every level input takes part in the backward (needs_grad checks plan.input only)
    plan.needs_grad = lambda v: v.act is not None
    anchor = det.__dict__.setdefault("_ym_anchor", torch.zeros(1, device=xs[0].device, requires_grad=True))
    xs32 = [x.float().contiguous() for x in xs]
    if torch.is_grad_enabled() and det.training:
        head = _DetectFn.apply(anchor, plan, *xs32)
    else:
        for v, x in zip(plan.inputs, xs32):
            v.act.t.copy_(x.permute(0, 2, 3, 1))
        plan.forward()
        plan.new_generation()
        head = plan.head.clone()
    return head, plan


def run_model(model, img: torch.Tensor):
    """Training-mode / eval-mode forward of the whole YOLOv11; returns the (B, A, 64+nc) fp32 head buffer."""
    if not img.is_cuda:
        raise YolomiError("yolomi kernels run on the MI355X only (got a CPU tensor)")
    B, C, H, W = img.shape
    ch = model.model[0].conv.in_channels
    if C != ch:
        # what the reference's first nn.Conv2d raises for a wrong plane count
        raise YolomiError(f"expected input[{B}, {C}, {H}, {W}] to have {ch} channels, but got {C} channels instead")
    key = ("model", B, H, W, model.training)
    cache = model.__dict__.setdefault("_ym_plans", {})
    pool = cache.setdefault(key, [])
    # the first plan of this shape whose activations no pending backward still needs (see Plan.pending)
    plan = next((p for p in pool if not p.pending), None)
    if plan is None:
        plan = Plan(model, B, H, W, img.device, model.training)
        plan.input_requires_grad = False
        plan.is_model = True
        lower_model(plan, model, (B, H, W))
        pool.append(plan)
    if model.training and torch.is_grad_enabled() and any(p_.pending for p_ in pool if p_ is not plan):
        # several forwards in flight THIS step: their gradients meet in .grad (install_grads adds), so data
        # parallelism all-reduces .grad after the backwards instead of each plan's buffer during its own.
        # A per-step flag (GradSync.sync clears it): the next ordinary step buckets again.
        model.__dict__["_ym_pooled_step"] = True
    if model.training:
        model.__dict__["_ym_last_plan"] = plan
    anchor = model.__dict__.setdefault("_ym_anchor", torch.zeros(1, device=img.device, requires_grad=True))
    img32 = img.float()
    if torch.is_grad_enabled() and model.training:
        head = _ModelFn.apply(img32, anchor, plan)
    else:
        plan.img = img32.contiguous()
        plan.forward()
        plan.new_generation()
        # a fresh tensor: the plan's buffer is rewritten by the next forward of this shape
        head = plan.head.clone()
    return head, plan
