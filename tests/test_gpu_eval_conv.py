"""ym_conv_fwd_eval — the eval-mode Conv block in one launch (conv -> BatchNorm with the running-statistics scale /
shift -> SiLU -> + residual, yolo11_modules.py:21-47 in eval mode) — vs a PyTorch fp32 reference of the same op, and
the eval forward of a whole model with it vs without it.

Kernel cases: the pipelined implicit GEMM's eval instance (>= 256 tiles), the halo-staged 3x3 kernel's C4 tile (20x20 /
10x10 maps, channel counts off the 32-channel chunk) and
the 2-stage implicit GEMM on 128x64 tiles (1x1, 3x3 stride 2, outputs narrower than the tile), each with the workspace
(the small-grid K-split: fp32 slices + a fold launch, where the policy splits) and without it (one launch), with and
without SiLU and a residual (its own strides at n > 1); the output is a
channel slice of a wider buffer (a concat slice: the other channels must stay untouched) and the residual a slice of
another buffer with the same strides.  The operands are rounded to the kernel's dtypes first (fp16 activations,
weights, residual), so the reference differs by fp32 accumulation order and the fp16 output rounding: rel 2e-3 of
max |y| (+1e-3).
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [
    # n, h, w, cin, cout, k, stride
    (1, 20, 20, 128, 128, 3, 1),
    (2, 20, 20, 72, 64, 3, 1),
    (1, 10, 10, 256, 128, 3, 1),
    (1, 20, 20, 512, 256, 1, 1),
    (2, 40, 40, 128, 128, 3, 2),
    (2, 13, 11, 64, 96, 3, 2),
    (1, 80, 80, 64, 64, 1, 1),
    (1, 160, 160, 32, 32, 3, 1),
    (2, 20, 20, 64, 40, 1, 1),
    (1, 20, 20, 136, 64, 3, 1),       # K-split: 27 K stages in 6 slices, slices starting inside a tap
    (1, 10, 10, 1024, 64, 1, 1),      # K-split of a 1x1: 16 stages in 4 slices
    (2, 40, 40, 48, 16, 3, 1),        # <= 32 output channels: the 128 x 32 eval tile (1 x 4 waves)
    (1, 20, 20, 256, 24, 3, 1),       # ... a ragged width on it, K-split (36 stages in 9 slices)
    (4, 128, 128, 64, 64, 1, 1),      # >= 256 tiles: the pipelined forward's eval instance (256 x 64 tile)
    (4, 128, 128, 128, 128, 3, 1),    # ... its 256 x 128 tile
]
PIPE_CASES = {(4, 128, 128, 64, 64, 1, 1), (4, 128, 128, 128, 128, 3, 1)}


def _desc(n, h, w, cin, cout, k, s, ld):
    from yolomi._lib import ConvDesc
    p = k // 2
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    d = ConvDesc()
    d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, oh, ow, cout, k, s, p
    d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * cin, cin, oh * ow * ld, ld
    d.out_f32, d.accumulate = 2, 0
    return d, oh, ow


@pytest.mark.parametrize("case", CASES, ids=[f"n{c[0]}h{c[1]}w{c[2]}c{c[3]}o{c[4]}k{c[5]}s{c[6]}" for c in CASES])
@pytest.mark.parametrize("act,with_res", [(1, False), (0, True), (1, True)])
@pytest.mark.parametrize("split", [True, False], ids=["ws", "nows"])
def test_conv_fwd_eval_vs_torch(case, act, with_res, split):
    from yolomi._lib import call, lib, stream_ptr
    n, h, w, cin, cout, k, s = case
    ld = cout + 24                                   # output / residual: channel slices of wider buffers
    d, oh, ow = _desc(n, h, w, cin, cout, k, s, ld)
    assert lib().ym_conv_fwd_eval_ok(ctypes.byref(d)) == 1, case
    assert (lib().ym_conv_algo(ctypes.byref(d), 0) == 2) == (case in PIPE_CASES), case
    g = torch.Generator().manual_seed(hash((case, act, with_res)) & 0xFFFF)
    x = torch.randn(n, h, w, cin, generator=g).half()
    wt = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).half()
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.2
    res = torch.randn(n, oh, ow, cout, generator=g).half() if with_res else None
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wt.float(), stride=s, padding=k // 2).permute(0, 2, 3, 1)
    ref = ref * scale + shift
    if act:
        ref = F.silu(ref)
    if res is not None:
        ref = ref + res.float()
    dev = torch.device("cuda")
    xd, wd = x.to(dev), wt.permute(0, 2, 3, 1).contiguous().to(dev)
    scd, shd = scale.to(dev), shift.to(dev)
    rld = cout + 40 if n > 1 else ld                  # a residual with its own strides, or the output's
    rbuf = torch.zeros(n, oh, ow, rld, dtype=torch.float16, device=dev)
    if res is not None:
        rbuf[..., 8:8 + cout] = res.to(dev)
    buf = torch.full((n, oh, ow, ld), 7.0, dtype=torch.float16, device=dev)
    # with the workspace: the K-split (two launches) where the grid is small; without it: one launch
    nws = lib().ym_conv_fwd_eval_workspace_size(ctypes.byref(d)) if split else 0
    ws = torch.full((max(nws, 1),), 255, dtype=torch.uint8, device=dev)     # NaN-filled: every slice element written
    torch.cuda.synchronize()
    call("ym_conv_fwd_eval", ctypes.byref(d), xd.data_ptr(), wd.data_ptr(), scd.data_ptr(), shd.data_ptr(), act,
         rbuf[..., 8:].data_ptr() if res is not None else None, oh * ow * rld, rld, buf[..., 8:].data_ptr(),
         ws.data_ptr() if nws else None, nws, stream_ptr(dev))
    torch.cuda.synchronize()
    out = buf.float().cpu()
    assert torch.all(out[..., :8] == 7.0) and torch.all(out[..., 8 + cout:] == 7.0), "channels outside the view written"
    y = out[..., 8:8 + cout]
    err, mag = float((y - ref).abs().max()), float(ref.abs().max())
    assert err <= 2e-3 * mag + 1e-3, f"max |diff| {err:.3e} vs max |ref| {mag:.3e}"


def test_conv_fwd_eval_ok_scope():
    """Not eval-epilogue cases at the default routing: a layer the halo-pipelined kernel takes, an accumulating or
    non-fp16 output."""
    from yolomi._lib import lib
    prev = lib().ym_conv_set_eval_route(-1)
    try:
        _ok_scope_default(lib())
    finally:
        lib().ym_conv_set_eval_route(prev)


def _ok_scope_default(L):
    lib = lambda: L                                             # noqa: E731
    d, _, _ = _desc(8, 160, 160, 64, 64, 3, 1, 64)              # the halo-pipelined 3x3 kernel (no eval instance)
    assert lib().ym_conv_fwd_eval_ok(ctypes.byref(d)) == 0
    d, _, _ = _desc(1, 20, 20, 64, 32, 1, 1, 32)                # 2-stage GEMM, 32 output channels (masked tile half)
    assert lib().ym_conv_fwd_eval_ok(ctypes.byref(d)) == 1
    d, _, _ = _desc(1, 20, 20, 256, 128, 1, 1, 128)
    assert lib().ym_conv_fwd_eval_ok(ctypes.byref(d)) == 1
    d.accumulate = 1
    assert lib().ym_conv_fwd_eval_ok(ctypes.byref(d)) == 0
    d.accumulate, d.out_f32 = 0, 1
    assert lib().ym_conv_fwd_eval_ok(ctypes.byref(d)) == 0
    assert lib().ym_conv_fwd_eval_workspace_size(ctypes.byref(d)) == 0


def test_conv_fwd_eval_split_policy():
    """K-split where a layer is <= 64 tiles with >= 12 K stages: ks = min(stages / 4, 256 / tiles, 16) fp32 slices of
    M x Cout; none with the setter at 0 or on a large grid."""
    from yolomi._lib import lib
    L = lib()
    prev_cfg, prev_split, prev_nk = L.ym_conv_set_eval_cfg(-1), L.ym_conv_set_eval_split(-1), L.ym_conv_set_eval_split_nk(-1)
    try:
        _split_policy_defaults(L)
    finally:
        L.ym_conv_set_eval_cfg(prev_cfg), L.ym_conv_set_eval_split(prev_split), L.ym_conv_set_eval_split_nk(prev_nk)


def _split_policy_defaults(L):
    d, _, _ = _desc(1, 20, 20, 256, 256, 3, 2, 256)            # 100 px x 256: 4 tiles, 36 stages -> 9 slices
    assert L.ym_conv_fwd_eval_workspace_size(ctypes.byref(d)) == 9 * 100 * 256 * 4
    d, _, _ = _desc(1, 80, 80, 128, 64, 3, 1, 64)              # 50 tiles, 18 stages -> 4 slices
    assert L.ym_conv_fwd_eval_workspace_size(ctypes.byref(d)) == 4 * 6400 * 64 * 4
    assert L.ym_conv_fwd_eval_ok(ctypes.byref(d)) == 1
    d, _, _ = _desc(16, 80, 80, 128, 64, 3, 1, 64)             # 800 tiles: one launch
    assert L.ym_conv_fwd_eval_workspace_size(ctypes.byref(d)) == 0
    d, _, _ = _desc(1, 20, 20, 256, 128, 1, 1, 128)            # 4 K stages: one launch
    assert L.ym_conv_fwd_eval_workspace_size(ctypes.byref(d)) == 0
    prev = L.ym_conv_set_eval_split(0)
    try:
        d, _, _ = _desc(1, 20, 20, 256, 256, 3, 2, 256)
        assert L.ym_conv_fwd_eval_workspace_size(ctypes.byref(d)) == 0
    finally:
        L.ym_conv_set_eval_split(prev)


@pytest.mark.parametrize("scale_name,imgsz,bs", [("s", 640, 1), ("n", 320, 2)])
def test_eval_forward_one_launch_blocks_vs_unfused(scale_name, imgsz, bs, monkeypatch):
    """The eval forward with the one-launch Conv blocks (default) against the same model with them off
    (YM_EVAL_FUSE=0: conv with an fp16 z, then ym_bn_apply): most blocks take the one-launch path at these sizes, and
    the outputs agree to fp16 rounding (the one-launch path normalises the fp32 accumulator instead of the fp16 z)."""
    import yaml
    from pathlib import Path
    from models import build_yolo11
    root = Path(__file__).resolve().parents[1] / "yolo-scratch_amd"
    cfg = yaml.safe_load((root / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = scale_name
    torch.manual_seed(7)
    m = build_yolo11(cfg, ch=1, nc=5).cuda().eval()
    img = torch.rand(bs, 1, imgsz, imgsz, generator=torch.Generator().manual_seed(8)).cuda()

    def run():
        with torch.no_grad():
            y, maps = m(img)
        torch.cuda.synchronize()
        return y.clone(), [t.clone() for t in maps]
    monkeypatch.setenv("YM_EVAL_GRAPH", "0")
    monkeypatch.setenv("YM_EVAL_FUSE", "0")
    y0, m0 = run()
    monkeypatch.setenv("YM_EVAL_FUSE", "1")
    y1, m1 = run()
    from yolomi.graph import ConvBN
    plan = next(iter(m.__dict__["_ym_plans"].values()))[0]
    convs = [op for op in plan.ops if type(op) is ConvBN]
    fused = [op for op in convs if op.__dict__.get("_evf", (0, None))[1] is not None]
    assert len(fused) >= len(convs) // 2, (len(fused), len(convs))
    for a, b in zip(m0, m1):
        err, mag = float((a - b).abs().max()), float(a.abs().max())
        assert err <= 2e-2 * mag + 1e-2, (err, mag)


@pytest.mark.parametrize("n,h,w,cout,act,ch", [(1, 64, 64, 32, 1, 1), (2, 37, 41, 16, 1, 1), (1, 20, 20, 64, 0, 1),
                                               (1, 30, 30, 96, 1, 1), (2, 33, 40, 32, 1, 3), (1, 24, 24, 256, 0, 4),
                                               (1, 17, 19, 16, 1, 2)])
def test_conv_first_fwd_eval_vs_torch(n, h, w, cout, act, ch):
    """ym_conv_first_fwd_eval — the stem Conv block (ch image planes -> cout, 3x3 s2 on the fp32 NCHW image) with the
    eval BatchNorm and SiLU in one launch, into a channel slice of a wider buffer, vs torch fp32 (fp16 output rounding)."""
    from yolomi._lib import call, stream_ptr
    g = torch.Generator().manual_seed(n * 1000 + h + cout)
    img = torch.rand(n, ch, h, w, generator=g)
    wt = torch.randn(cout, ch, 3, 3, generator=g) / (3 * ch ** 0.5)
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.2
    ref = F.conv2d(img, wt, stride=2, padding=1).permute(0, 2, 3, 1) * scale + shift
    if act:
        ref = F.silu(ref)
    oh, ow = ref.shape[1], ref.shape[2]
    ld = cout + 16
    dev = torch.device("cuda")
    buf = torch.full((n, oh, ow, ld), 7.0, dtype=torch.float16, device=dev)
    imgd, wd, scd, shd = img.to(dev), wt.to(dev), scale.to(dev), shift.to(dev)
    torch.cuda.synchronize()
    call("ym_conv_first_fwd_eval", imgd.data_ptr(), wd.data_ptr(), scd.data_ptr(), shd.data_ptr(), act,
         buf[..., 8:].data_ptr(), oh * ow * ld, ld, n, h, w, oh, ow, cout, 2, 1, ch, stream_ptr(dev))
    torch.cuda.synchronize()
    out = buf.float().cpu()
    assert torch.all(out[..., :8] == 7.0) and torch.all(out[..., 8 + cout:] == 7.0), "channels outside the view written"
    err, mag = float((out[..., 8:8 + cout] - ref).abs().max()), float(ref.abs().max())
    assert err <= 2e-3 * mag + 1e-3, f"max |diff| {err:.3e} vs max |ref| {mag:.3e}"


@pytest.mark.parametrize("n,h,w,heads,kd,hd,act,with_res", [(1, 20, 20, 4, 16, 32, 0, True), (2, 7, 9, 2, 8, 16, 1, False)])
def test_dw3x3_fwd_eval_vs_torch(n, h, w, heads, kd, hd, act, with_res):
    """ym_dw3x3_fwd_eval — Attention.pe (depthwise 3x3 on the v channels of qkv, channel map (c / hd) * (2kd + hd) + 2kd
    + c % hd) with the eval BatchNorm (+ SiLU) and + a residual view in one launch, vs torch fp32 (fp16 output rounding).
    The output and residual are channel slices of wider buffers."""
    from yolomi._lib import call, stream_ptr
    C, S = heads * hd, heads * (2 * kd + hd)
    g = torch.Generator().manual_seed(n * 100 + h + C)
    qkv = torch.randn(n, h, w, S, generator=g).half()
    wt = torch.randn(C, 1, 3, 3, generator=g) / 3
    scale = torch.rand(C, generator=g) + 0.5
    shift = torch.randn(C, generator=g) * 0.2
    res = torch.randn(n, h, w, C, generator=g).half() if with_res else None
    idx = torch.tensor([(c // hd) * (2 * kd + hd) + 2 * kd + c % hd for c in range(C)])
    v = qkv.float()[..., idx].permute(0, 3, 1, 2)
    ref = F.conv2d(v, wt, padding=1, groups=C).permute(0, 2, 3, 1) * scale + shift
    if act:
        ref = F.silu(ref)
    if res is not None:
        ref = ref + res.float()
    dev = torch.device("cuda")
    ld, rld = C + 16, C + 8
    buf = torch.full((n, h, w, ld), 7.0, dtype=torch.float16, device=dev)
    rbuf = torch.zeros(n, h, w, rld, dtype=torch.float16, device=dev)
    if res is not None:
        rbuf[..., 4:4 + C] = res.to(dev)
    qd, wd, scd, shd = qkv.to(dev), wt.reshape(C, 9).contiguous().to(dev), scale.to(dev), shift.to(dev)
    torch.cuda.synchronize()
    call("ym_dw3x3_fwd_eval", qd.data_ptr(), h * w * S, S, hd, 2 * kd + hd, 2 * kd, wd.data_ptr(), scd.data_ptr(),
         shd.data_ptr(), act, rbuf[..., 4:].data_ptr() if res is not None else None, h * w * rld, rld,
         buf[..., 8:].data_ptr(), h * w * ld, ld, n, h, w, C, stream_ptr(dev))
    torch.cuda.synchronize()
    out = buf.float().cpu()
    assert torch.all(out[..., :8] == 7.0) and torch.all(out[..., 8 + C:] == 7.0), "channels outside the view written"
    err, mag = float((out[..., 8:8 + C] - ref).abs().max()), float(ref.abs().max())
    assert err <= 2e-3 * mag + 1e-3, f"max |diff| {err:.3e} vs max |ref| {mag:.3e}"
