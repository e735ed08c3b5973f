"""Teacher-forced per-layer parity: EVERY op of a YOLOv11 training plan, forward and backward, against
the fp64 oracle evaluated on exactly that op's own inputs taken from the HIP run.

One training step of the real plan runs on the GPU (s@640 bs2, the headline network at its own
resolution, and m@256 bs1, the C4 graph).  Then, for every op, the oracle recomputes that op alone
from the HIP plan's own saved inputs — the fp16 activations the kernels read, the bf16 gradient that
arrived from the layers above, the fp32 master weights — so no error can compound across layers
(the whole-network tests in test_gpu_network.py bound the compounded result; this file pins each
layer).  Reference semantics per op (models/yolo11_modules.py):

* Conv (conv -> BatchNorm2d train -> SiLU | Identity, + Bottleneck / PSA residual, :21-47, :156-158):
  z = conv(x, W), BN batch statistics (biased variance, eps 1e-3), y; backward dz, dW, dgamma, dbeta,
  dx (the data-gradient kernel relaunched on the same dz into a zeroed buffer, so no other
  consumer's contribution is mixed in), and the running statistics (momentum 0.03, unbiased var);
* the stem Conv(1, c, 3, 2) on the fp32 image;
* Attention.pe (depthwise 3x3 + BN, :122, :134) on the v channels of qkv, + the attention output;
* the attention core (softmax(q^T k * kd^-0.5), v attn^T, :128-134): out and dq / dk / dv;
* SPPF's three chained 5x5 max-pools (:100-104) on the fp32 cv1 output: forward bit-exact, dx;
* Detect's bias 1x1 convs (:225, :232) writing the fp32 head rows: head values, dW, db, dx;
* nn.Upsample(2, 'nearest') and the PSA / C2PSA concat copies: bit-exact both ways.

Bounds (BASELINE north_star, 16-bit tensors): relative L2 <= 1e-2 for z, y, dz, dW, dgamma, dbeta, head
rows, attention out / dqkv and the running statistics; 2e-2 for dx.  A parameter whose whole
gradient is below 1e-6 of the plan's largest (a BN bias the loss sees only through a later
training-mode BN) is held in absolute terms on that scale instead.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_gpu_model import _seeded_model

pytestmark = pytest.mark.gpu

TOL, TOL_DX = 1e-2, 2e-2
D = torch.float64


def rel(a, b):
    a, b = torch.as_tensor(a).to(D).cpu(), torch.as_tensor(b).to(D).cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def vt(v, grad=False):
    """View (channel slice of an NHWC buffer) -> NCHW fp64 CPU tensor."""
    t = v.act.g if grad else v.act.t
    return t[..., v.c0:v.c0 + v.c].permute(0, 3, 1, 2).to(D).cpu()


def mat(t, B, H, W, as_fp16=False):
    """(M, C) pixel-major buffer -> NCHW fp64."""
    if as_fp16:
        t = t.view(torch.float16)
    return t.reshape(B, H, W, -1).permute(0, 3, 1, 2).to(D).cpu()


def bn_train(z, gamma, beta, eps):
    mean = z.mean((0, 2, 3))
    var = z.var((0, 2, 3), unbiased=False)
    xh = (z - mean[None, :, None, None]) / torch.sqrt(var + eps)[None, :, None, None]
    return gamma[None, :, None, None] * xh + beta[None, :, None, None], mean, z.var((0, 2, 3), unbiased=True)


class Report:
    def __init__(self):
        self.rows, self.fail = [], []

    def check(self, what, got, want, tol, scale=None, denom=None):
        if denom is not None:             # error relative to a stated scale (a statistic that may be ~0)
            e = float((torch.as_tensor(got).to(D) - torch.as_tensor(want).to(D)).norm()) / denom
        elif scale is not None and float(torch.as_tensor(want).norm()) < 1e-6 * scale:
            e = float((torch.as_tensor(got).to(D) - torch.as_tensor(want).to(D)).norm()) / scale
            tol = 1e-3
        else:
            e = rel(got, want)
        self.rows.append((e / tol, what, e))
        if not e <= tol:
            self.fail.append((what, e, tol))


def _relaunch_dgrad(op, dz_ptr, wt_ptr, desc, x_view, st):
    """The op's data-gradient kernel on its own dz into a zeroed copy of x's gradient buffer."""
    from yolomi._lib import call
    buf = torch.zeros_like(x_view.act.t, dtype=torch.bfloat16)
    acc = desc.accumulate
    desc.accumulate = 0
    call("ym_conv_dgrad", ctypes.byref(desc), dz_ptr, wt_ptr, buf.data_ptr() + 2 * x_view.c0, st)
    desc.accumulate = acc
    torch.cuda.synchronize()
    return buf[..., x_view.c0:x_view.c0 + x_view.c].permute(0, 3, 1, 2).to(D).cpu()


def kernel_of(desc, direction):
    """(id, name) of the conv kernel instance the library runs for desc (0 fwd, 1 dgrad, 2 wgrad)."""
    from yolomi._lib import lib
    buf = ctypes.create_string_buffer(96)
    kid = lib().ym_conv_kernel(ctypes.byref(desc), direction, buf, 96)
    return kid, buf.value.decode()


def conv_launches(plan):
    """Every implicit-GEMM conv launch of a training plan: (op index, direction, desc) for the ConvBN forwards,
    data gradients (where the input takes a gradient) and weight gradients, and Detect's bias 1x1 convs."""
    out = []
    for i, op in enumerate(plan.ops):
        kind = type(op).__name__
        if kind == "ConvBN":
            out += [(i, 0, op.desc), (i, 2, op.desc)]
            if plan.needs_grad(op.x):
                out.append((i, 1, op.desc))
        elif kind == "HeadLevel":
            for tag, df, db in (("box", op.fb, op.bb), ("cls", op.fc, op.bc)):
                out += [(f"{i}{tag}", 0, df), (f"{i}{tag}", 1, db), (f"{i}{tag}", 2, db)]
    return out


def selection_at(plan, n):
    """{(op, direction): (kernel id, name)} the library selects for this plan's convs with n images per batch
    (the same descriptors with n in place of the plan's batch; no override)."""
    from yolomi._lib import ConvDesc, lib
    prev = lib().ym_conv_set_select_batch(0)
    try:
        sel = {}
        for i, dr, d in conv_launches(plan):
            dn = ConvDesc.from_buffer_copy(d)
            dn.n = n
            sel[(i, dr)] = kernel_of(dn, dr)
        return sel
    finally:
        lib().ym_conv_set_select_batch(prev)


def teacher_forced(scale, imgsz, bs, seed):
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from yolomi._lib import call, stream_ptr
    from yolomi import graph as G

    m = _seeded_model(scale).train()
    state0 = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    b = {k: v.cuda() for k, v in synth_batch(bs, imgsz, seed=seed).items()}
    heads = m(b["img"])
    plan = m.__dict__["_ym_last_plan"]
    B = plan.B
    torch.cuda.synchronize()
    # forward state the backward overwrites (z -> dz in place) or that later forwards would
    snap = {i: (op.z.clone(), op.bnv.clone()) for i, op in enumerate(plan.ops) if getattr(op, "z", None) is not None}
    loss, _ = v8DetectionLoss(m)(heads, b)
    loss.backward()
    torch.cuda.synchronize()
    st = stream_ptr(plan.dev)
    gmax = max(float(p.grad.norm()) for p in m.parameters() if p.grad is not None)
    names = {id(p): k for k, p in m.named_parameters()}
    bufs = {k: v for k, v in m.named_buffers()}
    bnames = {id(v): k for k, v in bufs.items()}
    R = Report()
    R.kernels = {}                       # (op, direction) -> kernel (id, name) whose output was checked

    def seen(i, dr, d):
        R.kernels[(i, dr)] = kernel_of(d, dr)

    def pgrad(p):
        return plan.grad_view(p).to(D).cpu()

    for i, op in enumerate(plan.ops):
        kind = type(op).__name__
        tag = f"{i}:{kind}"
        if kind in ("ConvBN", "StemConvBN", "DWConvBN"):
            mod = op.m
            tag = f"{i}:{names[id(mod.conv.weight)][:-12]}"
            W = mod.conv.weight.detach().to(D).cpu().requires_grad_(True)
            gam = mod.bn.weight.detach().to(D).cpu().requires_grad_(True)
            bet = mod.bn.bias.detach().to(D).cpu().requires_grad_(True)
            eps = float(mod.bn.eps)
            oh, ow = op.y.H, op.y.W
            if kind == "StemConvBN":
                x = plan.img.to(D).cpu()
            elif kind == "DWConvBN":
                hd, hs, goff = op.map
                heads_n = op.C // hd
                q = vt(op.x)
                idx = torch.cat([torch.arange(h * hs + goff, h * hs + goff + hd) for h in range(heads_n)])
                x = q[:, idx]
            else:
                x = vt(op.x)
            x = x.requires_grad_(True)
            if kind == "DWConvBN":
                z = F.conv2d(x, W, stride=1, padding=1, groups=op.C)
            else:
                z = F.conv2d(x, W, stride=op.s, padding=op.k // 2)
            z.retain_grad()
            u, mean, var_u = bn_train(z, gam, bet, eps)
            y = F.silu(u) if op.act else u
            if op.res is not None:
                y = y + vt(op.res)
            z_h, bnv_h = snap[i]
            R.check(f"{tag} z", mat(z_h, B, oh, ow, as_fp16=True), z.detach(), TOL)
            if kind == "ConvBN":
                seen(i, 0, op.desc)
            R.check(f"{tag} y", vt(op.y), y.detach(), TOL)
            # batch means may sit near 0: their error is stated relative to the batch standard deviations
            sd = float(var_u.detach().sqrt().norm())
            R.check(f"{tag} bn mean", bnv_h[2].cpu(), mean.detach(), TOL, denom=sd)
            # running statistics: 0.97 * before + 0.03 * batch (unbiased variance), reference BN train
            rm0, rv0 = state0[bnames[id(mod.bn.running_mean)]], state0[bnames[id(mod.bn.running_var)]]
            R.check(f"{tag} running_mean", mod.bn.running_mean.cpu(), 0.97 * rm0.to(D) + 0.03 * mean.detach(), TOL,
                    denom=0.03 * sd)
            R.check(f"{tag} running_var", mod.bn.running_var.cpu(), 0.97 * rv0.to(D) + 0.03 * var_u.detach(), TOL)
            dy = vt(op.y, grad=True)
            y.backward(dy)
            if kind != "StemConvBN":          # the stem's fused backward never writes dz (ym_stem_bwd_wgrad_stored)
                R.check(f"{tag} dz", mat(op.z, B, oh, ow), z.grad, TOL)
            R.check(f"{tag} dW", pgrad(mod.conv.weight), W.grad, TOL, gmax)
            if kind == "ConvBN":
                seen(i, 2, op.desc)
            R.check(f"{tag} dgamma", pgrad(mod.bn.weight), gam.grad, TOL, gmax)
            R.check(f"{tag} dbeta", pgrad(mod.bn.bias), bet.grad, TOL, gmax)
            if kind == "ConvBN" and plan.needs_grad(op.x):
                dx = _relaunch_dgrad(op, op.z.data_ptr(), op.wt.data_ptr(), op.desc, op.x, st)
                R.check(f"{tag} dx", dx, x.grad, TOL_DX)
                seen(i, 1, op.desc)
            elif kind == "DWConvBN":
                from yolomi._lib import lib
                buf = torch.zeros_like(op.x.act.t, dtype=torch.bfloat16)
                dw = torch.zeros_like(mod.conv.weight)
                ws = torch.empty(max(lib().ym_dw3x3_bwd_workspace_size(op.C) // 4, 1), dtype=torch.float32,
                                 device=plan.dev)
                hd, hs, goff = op.map
                call("ym_dw3x3_bwd", op.x.ptr(), op.x.bs, op.x.ld, hd, hs, goff, mod.conv.weight.data_ptr(),
                     op.z.data_ptr(), buf.data_ptr() + 2 * op.x.c0, op.x.bs, op.x.ld, dw.data_ptr(), B, oh, ow, op.C, 0,
                     ws.data_ptr(), ws.numel() * 4, st)
                torch.cuda.synchronize()
                dq = buf[..., op.x.c0:op.x.c0 + op.x.c].permute(0, 3, 1, 2).to(D).cpu()
                R.check(f"{tag} dx(v)", dq[:, idx], x.grad, TOL_DX)
                R.check(f"{tag} dW relaunch", dw.cpu(), W.grad, TOL)
        elif kind == "HeadLevel":
            xb, xc = vt(op.xb).requires_grad_(True), vt(op.xc).requires_grad_(True)
            Wb = op.box.weight.detach().to(D).cpu().requires_grad_(True)
            bb = op.box.bias.detach().to(D).cpu().requires_grad_(True)
            Wc = op.cls.weight.detach().to(D).cpu().requires_grad_(True)
            bc = op.cls.bias.detach().to(D).cpu().requires_grad_(True)
            hb, hc = F.conv2d(xb, Wb, bb), F.conv2d(xc, Wc, bc)
            h = torch.cat((hb, hc), 1)                                   # (B, 64+nc, H, W)
            HW = op.HW
            rows = plan.head[:, op.a_off:op.a_off + HW, :].to(D).cpu()   # (B, HW, no)
            R.check(f"{tag} head rows", rows, h.detach().flatten(2).transpose(1, 2), TOL)
            dh = plan.dhead[:, op.a_off:op.a_off + HW, :].to(D).cpu().transpose(1, 2).reshape(h.shape)
            h.backward(dh)
            R.check(f"{tag} box dW", pgrad(op.box.weight), Wb.grad, TOL, gmax)
            R.check(f"{tag} box db", pgrad(op.box.bias), bb.grad, TOL, gmax)
            R.check(f"{tag} cls dW", pgrad(op.cls.weight), Wc.grad, TOL, gmax)
            R.check(f"{tag} cls db", pgrad(op.cls.bias), bc.grad, TOL, gmax)
            R.check(f"{tag} box dx", _relaunch_dgrad(op, op.dzb.data_ptr(), op.wb_t.data_ptr(), op.bb, op.xb, st),
                    xb.grad, TOL_DX)
            R.check(f"{tag} cls dx", _relaunch_dgrad(op, op.dzc.data_ptr(), op.wc_t.data_ptr(), op.bc, op.xc, st),
                    xc.grad, TOL_DX)
            for t_, df, db in (("box", op.fb, op.bb), ("cls", op.fc, op.bc)):
                seen(f"{i}{t_}", 0, df)
                seen(f"{i}{t_}", 1, db)
                seen(f"{i}{t_}", 2, db)
        elif kind == "AttnCore":
            qkv = vt(op.qkv)
            Bq, C, H, Wd = qkv.shape
            N, nh, kd, hd = H * Wd, op.heads, op.kd, op.hd
            qkv = qkv.reshape(Bq, nh, 2 * kd + hd, N).requires_grad_(True)
            q, k, v = qkv.split([kd, kd, hd], dim=2)
            att = ((q.transpose(-2, -1) @ k) * op.scale).softmax(-1)
            out = (v @ att.transpose(-2, -1)).reshape(Bq, nh * hd, H, Wd)
            R.check(f"{tag} out", vt(op.out), out.detach(), TOL)
            out.backward(vt(op.out, grad=True))
            buf = torch.zeros_like(op.qkv.act.t, dtype=torch.bfloat16)
            o = op.out
            call("ym_attn_bwd", op.qkv.ptr(), op.qkv.bs, op.qkv.ld, o.ptr(), o.bs, o.ld, o.gptr(), o.bs, o.ld,
                 op.lse.data_ptr(), B, nh, N, op.scale, op.ws.data_ptr(), buf.data_ptr() + 2 * op.qkv.c0, op.qkv.bs,
                 op.qkv.ld, 0, 0, 0, st)
            torch.cuda.synchronize()
            dqkv = buf[..., op.qkv.c0:op.qkv.c0 + op.qkv.c].permute(0, 3, 1, 2).to(D).cpu()
            R.check(f"{tag} dqkv", dqkv.reshape(qkv.shape), qkv.grad, TOL)
        elif kind == "SPPFPools":
            s0, s1, s2, s3 = op.slices
            p0 = op.P[0].reshape(B, op.H, op.W, op.C).permute(0, 3, 1, 2).to(D).cpu().requires_grad_(True)
            p1 = F.max_pool2d(p0, 5, 1, 2)
            p2 = F.max_pool2d(p1, 5, 1, 2)
            p3 = F.max_pool2d(p2, 5, 1, 2)
            for j, (pj, sj) in enumerate(((p1, s1), (p2, s2), (p3, s3))):
                hip = sj.act.t[..., sj.c0:sj.c0 + sj.c].permute(0, 3, 1, 2).cpu()
                want = pj.detach().to(torch.float32).to(hip.dtype)
                assert torch.equal(hip, want), f"{tag} pool {j + 1} not bit-exact"
            torch.autograd.backward([p1, p2, p3], [vt(s1, True), vt(s2, True), vt(s3, True)])
            buf = torch.zeros_like(s0.act.t, dtype=torch.bfloat16)
            call("ym_sppf_bwd", op.code.data_ptr(), s1.gptr(), s2.gptr(), s3.gptr(), s1.bs, s1.ld,
                 buf.data_ptr() + 2 * s0.c0, s0.bs, s0.ld, 0, None, B, op.H, op.W, op.C, st)
            torch.cuda.synchronize()
            R.check(f"{tag} dx", buf[..., s0.c0:s0.c0 + s0.c].permute(0, 3, 1, 2).to(D).cpu(), p0.grad, TOL)
        elif kind in ("Upsample2", "Copy"):
            x, y = vt(op.x), vt(op.y)
            want = F.interpolate(x, scale_factor=2, mode="nearest") if kind == "Upsample2" else x
            assert torch.equal(y, want), f"{tag} forward not bit-exact"
    R.plan = plan
    worst = sorted(R.rows)[-6:]
    print(f"{scale}@{imgsz} bs{bs}: {len(R.rows)} checks; worst err/tol", [(f"{r:.2f}", w, f"{e:.2e}") for r, w, e in worst])
    assert not R.fail, R.fail
    return R


@pytest.mark.parametrize("scale,imgsz,bs,select", [("s", 640, 2, 64), ("m", 256, 1, 0), ("x", 128, 1, 0)])
def test_teacher_forced_every_layer(scale, imgsz, bs, select):
    """select = 64: every conv kernel choice (kernel, template instance, tile) is made as for the bench's
    s@640 bs64 step (ym_conv_set_select_batch) while the batch is 2, so this test checks, op by op, exactly
    the kernels the benchmarked step runs — the direct / quad kernels on the persistent grids of the 160x160
    stem stage, the halo-pipelined, pipelined, halo and implicit-GEMM instances and every weight-gradient
    instance.  The set of (op, direction, kernel) the bs64 plan selects is computed from the plan's own
    descriptors and every element of it must have been checked.  select = 0: m@256 bs1 and x@128 bs1 at their own
    sizes (x: the 96-channel stem and the 384-channel depthwise pe run as channel pieces 64 + 32 / 256 + 128)."""
    from yolomi._lib import lib
    torch.set_num_threads(min(16, torch.get_num_threads()))
    prev = lib().ym_conv_set_select_batch(select)
    try:
        R = teacher_forced(scale, imgsz, bs, seed=31)
        # the override reproduces the bs64 choice launch by launch
        if select:
            want = selection_at(R.plan, select)
            got = {(i, dr): kernel_of(d, dr) for i, dr, d in conv_launches(R.plan)}
            assert got == want, sorted(set(got.items()) ^ set(want.items()))[:8]
        else:
            want = selection_at(R.plan, R.plan.B)
    finally:
        lib().ym_conv_set_select_batch(prev)
    missing = sorted(((str(k[0]), k[1]), v) for k, v in want.items() if R.kernels.get(k) != v)
    assert not missing, f"selected but not checked: {missing[:10]}"
    names = sorted({v[1] for v in want.values()})
    print(f"{scale}@{imgsz}: {len(want)} conv launches checked over {len(names)} kernel instances: {names}")
    if select == 64:
        # the instances the bs64 plan is known to run must be among them
        fams = {n.split(" ")[0] for n in names}
        assert {"direct", "hpipe", "pipe", "halo", "gemm", "wgrad3", "wgrad1"} <= fams, fams
    kinds = {w.split(" ")[0].split(":")[1] for _, w, _ in R.rows}
    assert any("model.0" in k for k in kinds)                   # the stem was checked
