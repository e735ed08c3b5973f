"""Implicit-GEMM conv kernels (fwd / dgrad / wgrad) vs a PyTorch fp32 reference of the same op.

The operands are rounded to the kernel's input dtypes first (fp16 activations and forward
weights, bf16 gradients and dgrad weights), so the reference differs from the kernel only
by fp32 accumulation order and the output rounding:
  fwd  fp32 out: rel 1e-3 of max|y|
  dgrad bf16 out: rel 1e-2 of max|dx| (one bf16 rounding = 2^-8)
  wgrad fp32 out: rel 1e-3 of max|dw| (x is converted fp16 -> bf16 at staging, mirrored here),
    OIHW, overwrite and accumulate; the 3x3 (all taps per block), 1x1 (flat pixels) and generic
    (here: 1x1 stride 2) kernels are all covered
Shapes cover odd spatial sizes, both strides, k = 1 and 3, channel counts that are not
multiples of the tile sizes, 8/16/32-channel inputs (taps packed into one K step), and the
4-parity-class stride-2 dgrad (a 1x1 stride-2 conv
leaves three of the classes with no tap: their gradient must be exactly zero).
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [
    # n, h, w, cin, cout, k, stride, pad
    (2, 9, 11, 64, 96, 3, 2, 1),
    (2, 8, 8, 32, 64, 3, 1, 1),
    (1, 7, 5, 48, 40, 1, 2, 0),
    (2, 13, 13, 128, 136, 3, 2, 1),
    (1, 6, 6, 16, 24, 1, 1, 0),
    (3, 20, 20, 256, 128, 3, 2, 1),
    (1, 5, 7, 520, 264, 3, 1, 1),
    (2, 9, 9, 256, 136, 1, 1, 0),
    (2, 33, 17, 64, 64, 3, 1, 1),
    # halo-staged 3x3 stride-1 kernel (conv_halo.hip): 16-wide tiles, whole-row tiles (20, 40, 10
    # wide), 8-wave 256x128 tiles, channel counts that are not multiples of the 32-channel chunk
    (2, 32, 32, 64, 128, 3, 1, 1),
    (5, 20, 20, 96, 64, 3, 1, 1),
    (1, 40, 40, 128, 136, 3, 1, 1),
    (16, 64, 64, 32, 128, 3, 1, 1),
    (3, 24, 10, 72, 80, 3, 1, 1),
    # weight gradient on whole-row units (wgrad.hip: 20 x 3 rows on 20-wide maps, stride 1 and 2;
    # 10 x 6 on 10-wide ones), with an odd unit count per split (a unit of zeros pads the pair)
    (2, 40, 40, 128, 72, 3, 2, 1),
    (1, 20, 20, 64, 64, 3, 1, 1),
    # maps >= 64 wide: two register sets (units t+1, t+2 in flight), 7 units per split (odd)
    (3, 64, 72, 64, 64, 3, 1, 1),
    # narrow inputs: several taps share one 64-deep K step (fwd Kin = cin, dgrad Kin = cout)
    (2, 9, 7, 64, 32, 3, 1, 1),
    (1, 10, 10, 8, 16, 3, 1, 1),
    (2, 11, 11, 16, 32, 3, 2, 1),
]


def _desc(n, h, w, cin, cout, k, s, p):
    from yolomi._lib import ConvDesc
    oh = (h + 2 * p - k) // s + 1
    ow = (w + 2 * p - k) // s + 1
    d = ConvDesc()
    d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, oh, ow, cout, k, s, p
    d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * cin, cin, oh * ow * cout, cout
    d.out_f32, d.accumulate = 1, 0
    return d, oh, ow


@pytest.fixture(params=["auto", "halo"])
def halo_mode(request):
    """Run each shape under the default kernel selection and with the halo kernel wherever it applies."""
    from yolomi._lib import lib
    prev = lib().ym_conv_set_halo(-1 if request.param == "auto" else 1)
    yield request.param
    lib().ym_conv_set_halo(prev)


@pytest.mark.parametrize("shape", SHAPES, ids=[f"n{s[0]}h{s[1]}w{s[2]}c{s[3]}o{s[4]}k{s[5]}s{s[6]}" for s in SHAPES])
def test_conv_kernels_vs_torch(shape, halo_mode):
    from yolomi._lib import call
    n, h, w, cin, cout, k, s, p = shape
    d, oh, ow = _desc(*shape)
    g = torch.Generator().manual_seed(hash(shape) & 0xFFFF)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, h, w, cin, generator=g).half()
    wt = (torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5)
    dz = torch.randn(n, oh, ow, cout, generator=g).bfloat16()

    w16 = wt.half()                                   # forward copy [cout][kh][kw][cin] fp16
    wbf = wt.bfloat16()                               # dgrad copy [cin][kh][kw][cout] bf16
    xd = x.to(dev)
    w_fwd = w16.permute(0, 2, 3, 1).contiguous().to(dev)
    w_t = wbf.permute(1, 2, 3, 0).contiguous().to(dev)
    dzd = dz.to(dev)
    st = torch.cuda.current_stream().cuda_stream

    # forward, fp32 output
    y = torch.empty(n, oh, ow, cout, dtype=torch.float32, device=dev)
    call("ym_conv_fwd", ctypes.byref(d), xd.data_ptr(), w_fwd.data_ptr(), y.data_ptr(), None, None, None, st)
    x_nchw = x.float().permute(0, 3, 1, 2)
    y_ref = F.conv2d(x_nchw, w16.float(), stride=s, padding=p).permute(0, 2, 3, 1)
    # dgrad, bf16 output; prefill with garbage: every pixel must be written
    dx = torch.full((n, h, w, cin), float("nan"), dtype=torch.bfloat16, device=dev)
    call("ym_conv_dgrad", ctypes.byref(d), dzd.data_ptr(), w_t.data_ptr(), dx.data_ptr(), st)
    dz_nchw = dz.float().permute(0, 3, 1, 2)
    dx_ref = torch.nn.grad.conv2d_input((n, cin, h, w), wbf.float(), dz_nchw, stride=s, padding=p).permute(0, 2, 3, 1)
    # wgrad: OIHW fp32, split-K partials in the workspace; then accumulate=1 adds a second copy
    from yolomi._lib import lib
    ws = torch.empty(max(lib().ym_conv_wgrad_workspace_size(ctypes.byref(d)) // 4, 1), dtype=torch.float32, device=dev)
    dw = torch.full((cout, cin, k, k), float("nan"), dtype=torch.float32, device=dev)
    call("ym_conv_wgrad", ctypes.byref(d), dzd.data_ptr(), xd.data_ptr(), ws.data_ptr(), ws.numel() * 4,
         dw.data_ptr(), 0, st)
    dw2 = dw.clone()
    call("ym_conv_wgrad", ctypes.byref(d), dzd.data_ptr(), xd.data_ptr(), ws.data_ptr(), ws.numel() * 4,
         dw2.data_ptr(), 1, st)
    dw_ref = torch.nn.grad.conv2d_weight(x.bfloat16().float().permute(0, 3, 1, 2), (cout, cin, k, k), dz_nchw,
                                         stride=s, padding=p)
    torch.cuda.synchronize()

    def rel(a, b):
        return float((a.float().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-12))

    assert rel(y, y_ref) < 1e-3
    assert torch.isfinite(dx.float()).all()
    assert rel(dx, dx_ref) < 1e-2
    assert rel(dw, dw_ref) < 1e-3
    assert rel(dw2, 2 * dw_ref) < 1e-3
    if k == 1 and s == 2:
        # pixels at odd rows or odd columns receive no tap
        dxc = dx.float().cpu()
        assert (dxc[:, 1::2] == 0).all() and (dxc[:, :, 1::2] == 0).all()


HALO = [(2, 32, 32, 64, 128, 3, 1, 1), (5, 20, 20, 96, 64, 3, 1, 1), (1, 40, 40, 128, 136, 3, 1, 1),
        (16, 64, 64, 32, 128, 3, 1, 1), (3, 24, 10, 72, 80, 3, 1, 1), (2, 33, 17, 64, 64, 3, 1, 1)]


def test_halo_kernel_selected(halo_mode):
    """The 3x3 stride-1 shapes above with >= 64 output channels run the halo kernel (fwd) when forced;
    by default maps <= 48 wide or with <= 64 output channels do (rule 3), rule 2 only maps <= 24 wide."""
    from yolomi._lib import lib
    if halo_mode == "auto":
        d, _, _ = _desc(5, 20, 20, 96, 64, 3, 1, 1)
        assert lib().ym_conv_algo(ctypes.byref(d), 0) == 1
        d, _, _ = _desc(1, 40, 40, 128, 136, 3, 1, 1)
        assert lib().ym_conv_algo(ctypes.byref(d), 0) == 1
        d, _, _ = _desc(1, 56, 56, 128, 136, 3, 1, 1)
        assert lib().ym_conv_algo(ctypes.byref(d), 0) == 0
        prev = lib().ym_conv_set_halo(2)
        try:
            d, _, _ = _desc(1, 40, 40, 128, 136, 3, 1, 1)
            assert lib().ym_conv_algo(ctypes.byref(d), 0) == 0
        finally:
            lib().ym_conv_set_halo(prev)
        return
    for shape in HALO:
        d, _, _ = _desc(*shape)
        assert lib().ym_conv_algo(ctypes.byref(d), 0) == 1, shape
    d, _, _ = _desc(2, 32, 32, 64, 128, 3, 1, 1)
    assert lib().ym_conv_algo(ctypes.byref(d), 1) == 1          # dgrad: 64 output channels
    d, _, _ = _desc(2, 9, 11, 64, 96, 3, 2, 1)
    assert lib().ym_conv_algo(ctypes.byref(d), 0) == 0          # stride 2: implicit GEMM


def test_dgrad_accumulate_stride2():
    """accumulate=1 adds the transposed conv into an existing gradient (concat/residual fan-in)."""
    from yolomi._lib import call
    shape = (2, 10, 12, 64, 64, 3, 2, 1)
    n, h, w, cin, cout, k, s, p = shape
    d, oh, ow = _desc(*shape)
    d.accumulate = 1
    g = torch.Generator().manual_seed(7)
    dev = torch.device("cuda", 0)
    wt = torch.randn(cout, cin, k, k, generator=g) * 0.05
    wbf = wt.bfloat16()
    dz = torch.randn(n, oh, ow, cout, generator=g).bfloat16()
    base = torch.randn(n, h, w, cin, generator=g).bfloat16()
    dx = base.to(dev)
    w_t = wbf.permute(1, 2, 3, 0).contiguous().to(dev)
    dzd = dz.to(dev)
    call("ym_conv_dgrad", ctypes.byref(d), dzd.data_ptr(), w_t.data_ptr(), dx.data_ptr(),
         torch.cuda.current_stream().cuda_stream)
    ref = base.float() + torch.nn.grad.conv2d_input((n, cin, h, w), wbf.float(), dz.float().permute(0, 3, 1, 2),
                                                    stride=s, padding=p).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    err = float((dx.float().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 1e-2


# persistent pipelined implicit GEMM (conv_pipe.hip), forced on with ym_conv_set_pipe(2) (layers of
# >= 256 tiles): 256 x 128 tiles (>= 128 output channels) and 256 x 64 tiles, 3x3 and 1x1, stride 2
# forward and the 4-class stride-2 data gradient, partial pixel / channel tiles, strided channel views
# (a conv reading / writing a slice of a concat buffer), fp16 + BN statistics / bf16 outputs, and
# gradient accumulation
PIPE = [
    # n, h, w, cin, cout, k, stride, pad, in_extra, out_extra (extra channels of the surrounding view)
    (16, 64, 64, 128, 128, 3, 1, 1, 0, 0),
    (18, 61, 63, 128, 192, 3, 1, 1, 64, 8),
    (16, 64, 64, 64, 128, 3, 1, 1, 0, 64),
    (16, 128, 128, 64, 128, 3, 2, 1, 0, 0),
    (70, 63, 61, 128, 128, 3, 2, 1, 0, 0),     # odd map: unequal stride-2 classes (class-major tile order)
    (16, 64, 64, 256, 128, 1, 1, 0, 128, 0),
    (12, 80, 80, 64, 64, 3, 1, 1, 0, 0),
]


@pytest.mark.parametrize("shape", PIPE, ids=[f"n{s[0]}h{s[1]}w{s[2]}c{s[3]}o{s[4]}k{s[5]}s{s[6]}" for s in PIPE])
def test_pipe_kernel_vs_torch(shape):
    """fp16 forward (+ BN statistic partials), bf16 data gradient (overwrite, then accumulate).  (The round-6
    32x32x16-MFMA and reads-first variants, measurement library only, passed this test on every shape:
    profiles/r06/pytest_pipe_variants.log.)"""
    from yolomi._lib import lib
    _views_fwd_dgrad_check(shape, lib().ym_conv_set_pipe, 2, 2)


# halo-staged PIPELINED 3x3 stride-1 kernel (conv_hpipe.hip), forced on with ym_conv_set_hpipe(2): 16x16-pixel
# tiles on maps whose sides are multiples of 16, 128-channel tiles (a partial second channel tile at 192),
# 2-4 input chunks of 64 channels, channel-slice views in and out, fp16 z + BN statistic partials,
# bf16 data gradient overwrite and accumulate
HPIPE = [
    (2, 16, 16, 128, 128, 3, 1, 1, 0, 0),
    (1, 32, 48, 128, 128, 3, 1, 1, 64, 0),
    (2, 16, 32, 128, 192, 3, 1, 1, 0, 8),
    (3, 32, 32, 256, 128, 3, 1, 1, 0, 0),
    (2, 48, 16, 192, 256, 3, 1, 1, 32, 64),
    (9, 80, 80, 128, 128, 3, 1, 1, 0, 0),
    # 64 -> 64: the 72 KB weight tensor resident in LDS (cfg 2), a halo per tile
    (2, 16, 16, 64, 64, 3, 1, 1, 0, 0),
    (3, 32, 48, 64, 64, 3, 1, 1, 64, 32),
    (9, 80, 80, 64, 64, 3, 1, 1, 0, 0),
]


@pytest.mark.parametrize("shape", HPIPE, ids=[f"n{s[0]}h{s[1]}w{s[2]}c{s[3]}o{s[4]}x{s[8]}y{s[9]}" for s in HPIPE])
def test_hpipe_kernel_vs_torch(shape):
    from yolomi._lib import lib
    _views_fwd_dgrad_check(shape, lib().ym_conv_set_hpipe, 2, 4)


def test_hpipe_selection():
    """By default the halo-pipelined kernel takes the 64 -> 64 3x3 stride-1 convs (weights resident in LDS) on
    16-multiple maps with >= 512 tiles (the 80x80 / 160x160 layers at bs64), in either direction; the >= 128-
    output-channel layers run the pipelined implicit GEMM (faster since round 4); never stride 2 or other maps."""
    from yolomi._lib import lib

    def desc(*shape):
        d, _, _ = _desc(*shape)
        d.out_f32 = 2                    # a Conv block's fp16 z
        return d
    d = desc(64, 80, 80, 128, 128, 3, 1, 1)
    assert lib().ym_conv_algo(ctypes.byref(d), 0) == 2 and lib().ym_conv_algo(ctypes.byref(d), 1) == 2
    d = desc(64, 80, 80, 128, 64, 3, 1, 1)
    assert lib().ym_conv_algo(ctypes.byref(d), 0) != 4 and lib().ym_conv_algo(ctypes.byref(d), 1) != 4
    d = desc(64, 80, 80, 64, 64, 3, 1, 1)
    assert lib().ym_conv_algo(ctypes.byref(d), 0) == 4 and lib().ym_conv_algo(ctypes.byref(d), 1) == 4
    for shape in [(64, 40, 40, 128, 128, 3, 1, 1), (64, 160, 160, 64, 64, 3, 2, 1), (2, 80, 80, 128, 128, 3, 1, 1),
                  (64, 80, 80, 32, 64, 3, 1, 1)]:
        d = desc(*shape)
        assert lib().ym_conv_algo(ctypes.byref(d), 0) != 4, shape


# halo-staged 3x3 kernel forced on (ym_conv_set_halo(1)) through the same training-path outputs the
# network uses: fp16 z + BN statistics, bf16 data gradient overwrite and accumulate (concat fan-in),
# channel-slice views, 16-wide and whole-row tiles, single-tile images (bs1 16x16: the s@128 network)
HALO_VIEWS = [
    (1, 16, 16, 64, 64, 3, 1, 1, 0, 0),
    (1, 32, 32, 128, 128, 3, 1, 1, 64, 0),
    (2, 20, 20, 128, 128, 3, 1, 1, 0, 128),
    (3, 40, 40, 64, 64, 3, 1, 1, 32, 32),
    (2, 16, 16, 256, 128, 3, 1, 1, 0, 0),
    (4, 80, 80, 64, 64, 3, 1, 1, 0, 0),
]


@pytest.mark.parametrize("shape", HALO_VIEWS,
                         ids=[f"n{s[0]}h{s[1]}w{s[2]}c{s[3]}o{s[4]}x{s[8]}y{s[9]}" for s in HALO_VIEWS])
def test_halo_kernel_views_vs_torch(shape):
    from yolomi._lib import lib
    pp, pd = lib().ym_conv_set_pipe(0), lib().ym_conv_set_direct(0)
    try:
        _views_fwd_dgrad_check(shape, lib().ym_conv_set_halo, 1, 1)
    finally:
        lib().ym_conv_set_pipe(pp)
        lib().ym_conv_set_direct(pd)


def _views_fwd_dgrad_check(shape, setter, mode, algo):
    """Forward (fp16 z + BN statistic partials) and data gradient (bf16, overwrite then accumulate)
    of one conv through channel-slice views, with kernel `algo` forced on by setter(mode)."""
    from yolomi._lib import call, lib, ConvDesc
    n, h, w, cin, cout, k, s, p, xe, ye = shape
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    d = ConvDesc()
    d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, oh, ow, cout, k, s, p
    d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * (cin + xe), cin + xe, oh * ow * (cout + ye), cout + ye
    d.out_f32, d.accumulate = 2, 0
    g = torch.Generator().manual_seed(hash(shape) & 0xFFFF)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, h, w, cin, generator=g).half()
    wt = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    dz = torch.randn(n, oh, ow, cout, generator=g).bfloat16()
    w16, wbf = wt.half(), wt.bfloat16()
    prev = setter(mode)
    try:
        assert lib().ym_conv_algo(ctypes.byref(d), 0) == algo
        assert lib().ym_conv_algo(ctypes.byref(d), 1) == algo
        xbuf = torch.zeros(n, h, w, cin + xe, dtype=torch.float16, device=dev)
        xbuf[..., :cin] = x.to(dev)
        ybuf = torch.full((n, oh, ow, cout + ye), 7.0, dtype=torch.float16, device=dev)
        rows = lib().ym_conv_fwd_stat_rows(ctypes.byref(d))
        ss = torch.full((rows, cout), float("nan"), device=dev)
        sq = torch.full((rows, cout), float("nan"), device=dev)
        st = torch.cuda.current_stream().cuda_stream
        w_fwd = w16.permute(0, 2, 3, 1).contiguous().to(dev)
        call("ym_conv_fwd", ctypes.byref(d), xbuf.data_ptr(), w_fwd.data_ptr(), ybuf.data_ptr(), None,
             ss.data_ptr(), sq.data_ptr(), st)
        # dgrad: dz in the output view, dx into the input view (overwrite, then accumulate a second copy)
        dzbuf = torch.zeros(n, oh, ow, cout + ye, dtype=torch.bfloat16, device=dev)
        dzbuf[..., :cout] = dz.to(dev)
        dxbuf = torch.full((n, h, w, cin + xe), float("nan"), dtype=torch.bfloat16, device=dev)
        dxbuf[..., cin:] = 3.0
        w_t = wbf.permute(1, 2, 3, 0).contiguous().to(dev)
        dd = ConvDesc.from_buffer_copy(d)
        call("ym_conv_dgrad", ctypes.byref(dd), dzbuf.data_ptr(), w_t.data_ptr(), dxbuf.data_ptr(), st)
        dx1 = dxbuf.clone()
        dd.accumulate = 1
        call("ym_conv_dgrad", ctypes.byref(dd), dzbuf.data_ptr(), w_t.data_ptr(), dxbuf.data_ptr(), st)
        torch.cuda.synchronize()
    finally:
        setter(prev)
    y_ref = F.conv2d(x.float().permute(0, 3, 1, 2), w16.float(), stride=s, padding=p).permute(0, 2, 3, 1)
    dx_ref = torch.nn.grad.conv2d_input((n, cin, h, w), wbf.float(), dz.float().permute(0, 3, 1, 2),
                                        stride=s, padding=p).permute(0, 2, 3, 1)

    def rel(a, b):
        return float((a.float().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-12))

    yc = ybuf.cpu()
    assert rel(yc[..., :cout], y_ref) < 2e-3                       # one fp16 rounding
    assert (yc[..., cout:] == 7.0).all()                           # the rest of the view untouched
    ref_sum, ref_sq = y_ref.reshape(-1, cout).sum(0), (y_ref.reshape(-1, cout) ** 2).sum(0)
    # per-channel sums can cancel to ~0: bound by the sum of magnitudes
    assert float((ss.sum(0).cpu() - ref_sum).abs().max()) < 1e-4 * float(y_ref.abs().reshape(-1, cout).sum(0).max())
    assert rel(sq.sum(0), ref_sq) < 1e-3
    d1 = dx1.float().cpu()
    assert torch.isfinite(d1).all()
    assert rel(d1[..., :cin], dx_ref) < 1e-2
    assert (d1[..., cin:] == 3.0).all()
    assert rel(dxbuf[..., :cin], 2 * dx_ref) < 1e-2


# direct register-weight kernel (conv_direct.hip), forced on at any size with ym_conv_set_direct(2):
# every instantiated (Cin, Cout, k, stride) in both directions, odd map sizes (partial 16-pixel groups,
# odd stride-2 parity classes), channel-slice views, fp16 + BN statistics forward, bf16 data gradient
# overwrite and accumulate
DIRECT = [
    # n, h, w, cin, cout, k, stride, in_extra, out_extra
    (2, 17, 19, 32, 64, 3, 2, 0, 0),
    (3, 33, 21, 32, 32, 3, 1, 32, 16),
    (2, 15, 13, 64, 64, 1, 1, 0, 64),
    (2, 11, 23, 96, 128, 1, 1, 32, 0),
    (1, 19, 9, 64, 64, 1, 1, 0, 0),
    (2, 21, 16, 32, 64, 3, 2, 32, 0),
    # >= 1 M input pixels: more tasks than the chip holds workgroups, so the persistent grid (CUs x occupancy)
    # is the resident cap and every workgroup runs many tasks (the BN partial rows = that grid)
    (10, 320, 320, 32, 64, 3, 2, 0, 0),
]


@pytest.mark.parametrize("shape", DIRECT, ids=[f"n{s[0]}h{s[1]}w{s[2]}c{s[3]}o{s[4]}k{s[5]}s{s[6]}" for s in DIRECT])
def test_direct_kernel_vs_torch(shape):
    """The direct register-weight kernel forced on (the stride-2 data gradient over 2x2-pixel quads, all four
    output-parity classes per task; odd maps leave partial quads) vs PyTorch fp32 on the same rounded operands."""
    from yolomi._lib import call, lib, ConvDesc
    n, h, w, cin, cout, k, s, xe, ye = shape
    p = k // 2
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    d = ConvDesc()
    d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, oh, ow, cout, k, s, p
    d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * (cin + xe), cin + xe, oh * ow * (cout + ye), cout + ye
    d.out_f32, d.accumulate = 2, 0
    g = torch.Generator().manual_seed(hash(shape) & 0xFFFF)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, h, w, cin, generator=g).half()
    wt = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    dz = torch.randn(n, oh, ow, cout, generator=g).bfloat16()
    w16, wbf = wt.half(), wt.bfloat16()
    prev = lib().ym_conv_set_direct(2)
    try:
        assert lib().ym_conv_algo(ctypes.byref(d), 0) == 3
        assert lib().ym_conv_algo(ctypes.byref(d), 1) == 3
        xbuf = torch.zeros(n, h, w, cin + xe, dtype=torch.float16, device=dev)
        xbuf[..., :cin] = x.to(dev)
        ybuf = torch.full((n, oh, ow, cout + ye), 7.0, dtype=torch.float16, device=dev)
        rows = lib().ym_conv_fwd_stat_rows(ctypes.byref(d))
        if n * oh * ow >= 1 << 18:
            # resident-capped persistent grid: CUs (256 on MI355X) x 1 or 2 workgroups per CU, far fewer than
            # the 16-pixel tasks (so each workgroup strides over many)
            assert rows in (256, 512) and rows * 64 < n * oh * ow // 16, rows
        ss = torch.full((rows, cout), float("nan"), device=dev)
        sq = torch.full((rows, cout), float("nan"), device=dev)
        st = torch.cuda.current_stream().cuda_stream
        w_fwd = w16.permute(0, 2, 3, 1).contiguous().to(dev)
        call("ym_conv_fwd", ctypes.byref(d), xbuf.data_ptr(), w_fwd.data_ptr(), ybuf.data_ptr(), None,
             ss.data_ptr(), sq.data_ptr(), st)
        dzbuf = torch.zeros(n, oh, ow, cout + ye, dtype=torch.bfloat16, device=dev)
        dzbuf[..., :cout] = dz.to(dev)
        dxbuf = torch.full((n, h, w, cin + xe), float("nan"), dtype=torch.bfloat16, device=dev)
        dxbuf[..., cin:] = 3.0
        w_t = wbf.permute(1, 2, 3, 0).contiguous().to(dev)
        call("ym_conv_dgrad", ctypes.byref(d), dzbuf.data_ptr(), w_t.data_ptr(), dxbuf.data_ptr(), st)
        dx1 = dxbuf.clone()
        dd = ConvDesc.from_buffer_copy(d)
        dd.accumulate = 1
        call("ym_conv_dgrad", ctypes.byref(dd), dzbuf.data_ptr(), w_t.data_ptr(), dxbuf.data_ptr(), st)
        torch.cuda.synchronize()
    finally:
        lib().ym_conv_set_direct(prev)
    y_ref = F.conv2d(x.float().permute(0, 3, 1, 2), w16.float(), stride=s, padding=p).permute(0, 2, 3, 1)
    dx_ref = torch.nn.grad.conv2d_input((n, cin, h, w), wbf.float(), dz.float().permute(0, 3, 1, 2),
                                        stride=s, padding=p).permute(0, 2, 3, 1)

    def rel(a, b):
        return float((a.float().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-12))

    yc = ybuf.cpu()
    assert rel(yc[..., :cout], y_ref) < 2e-3
    assert (yc[..., cout:] == 7.0).all()
    yr = y_ref.reshape(-1, cout)
    assert float((ss.sum(0).cpu() - yr.sum(0)).abs().max()) < 1e-4 * float(yr.abs().sum(0).max())
    assert rel(sq.sum(0), (yr ** 2).sum(0)) < 1e-3
    d1 = dx1.float().cpu()
    assert torch.isfinite(d1).all()
    assert rel(d1[..., :cin], dx_ref) < 1e-2
    assert (d1[..., cin:] == 3.0).all()
    assert rel(dxbuf[..., :cin], 2 * dx_ref) < 1e-2


@pytest.mark.parametrize("k,out_f32", [(3, 2), (3, 0), (1, 2)])
def test_conv_fwd_bias_on_every_policy(k, out_f32):
    """y = conv(x, w) + bias on a layer the halo-pipelined / direct kernels would take (3x3 stride 1, 80x80,
    128 channels; those kernels have no bias term): with every policy forced on, ym_conv_fwd must still add the
    bias (it routes a conv with bias to the kernels that have one).  vs PyTorch fp32 on the same rounded operands."""
    from yolomi._lib import call, lib, ConvDesc
    n, h, w, cin, cout, p = 2, 80, 80, 128, 128, k // 2
    d = ConvDesc()
    d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, h, w, cout, k, 1, p
    d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * cin, cin, h * w * cout, cout
    d.out_f32, d.accumulate = out_f32, 0
    g = torch.Generator().manual_seed(7 + k)
    dev = torch.device("cuda", 0)
    x = torch.randn(n, h, w, cin, generator=g).half()
    wt = (torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5).half()
    bias = torch.randn(cout, generator=g) * 4
    L = lib()
    prev = (L.ym_conv_set_hpipe(2), L.ym_conv_set_direct(2), L.ym_conv_set_pipe(2), L.ym_conv_set_halo(1))
    try:
        y = torch.zeros(n, h, w, cout, dtype=torch.float16 if out_f32 == 2 else torch.bfloat16, device=dev)
        # device copies held in names: a temporary's block returns to the caching allocator as soon as its
        # data_ptr() is taken, and the next argument's copy can land in it (round 5: x overwritten by the bias)
        xd, wd, bd = x.to(dev), wt.permute(0, 2, 3, 1).contiguous().to(dev), bias.to(dev)
        call("ym_conv_fwd", ctypes.byref(d), xd.data_ptr(), wd.data_ptr(), y.data_ptr(), bd.data_ptr(), None, None,
             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        L.ym_conv_set_hpipe(prev[0]); L.ym_conv_set_direct(prev[1]); L.ym_conv_set_pipe(prev[2]); L.ym_conv_set_halo(prev[3])
    ref = (F.conv2d(x.float().permute(0, 3, 1, 2), wt.float(), bias, padding=p)).permute(0, 2, 3, 1)
    err = float((y.float().cpu() - ref).abs().max() / ref.abs().max())
    assert err < (2e-3 if out_f32 == 2 else 1e-2), err


# ym_conv_fwd_bn: conv forward + BatchNorm finalize, the finalize folded into the pipelined / halo kernel's tail where
# ym_conv_fwd_bn_fused says so (tickets per channel tile, fixed-order fp64 fold), else conv + ym_bn_finalize.
# Both against the two-call path (ym_conv_fwd, ym_bn_finalize): z bit-identical, the coefficients and running
# statistics to 1e-6 (the fold order differs), num_batches_tracked +1 exactly; three calls in a row (the tickets
# re-arm themselves).
FOLD = [
    (16, 64, 64, 128, 128, 3, 1),      # pipe 256x128, one channel tile, fused
    (16, 64, 64, 256, 192, 1, 0),      # pipe 1x1, 2 channel tiles (192 = 128 + 64), fused
    (16, 128, 128, 64, 128, 3, 1),     # stride 1 128-channel: pipe
    (2, 20, 20, 128, 128, 3, 1),       # small map: halo-staged kernel (C8), fused
    (3, 20, 20, 64, 64, 3, 1),         # halo C4 (64-channel tiles), fused
    (2, 20, 20, 256, 128, 1, 0),       # small 1x1: 2-stage implicit GEMM, fused
    (24, 80, 80, 64, 64, 3, 1),        # halo-pipelined 64 -> 64 (weights resident, >= 512 tiles): not fused
]


@pytest.mark.parametrize("shape", FOLD, ids=[f"n{s[0]}h{s[1]}c{s[3]}o{s[4]}k{s[5]}" for s in FOLD])
def test_conv_fwd_bn_fold_matches_two_calls(shape):
    from yolomi._lib import BnFold, ConvDesc, call, lib
    n, h, w, cin, cout, k, p = shape
    d = ConvDesc()
    d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, h, w, cout, k, 1, p
    d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * cin, cin, h * w * cout, cout
    d.out_f32, d.accumulate = 2, 0
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, h, w, cin, generator=g).half().to(dev)
    wt = (torch.randn(cout, k, k, cin, generator=g) * (2.0 / (cin * k * k)) ** 0.5).half().to(dev)
    gamma = (1 + 0.1 * torch.randn(cout, generator=g)).to(dev)
    beta = (0.1 * torch.randn(cout, generator=g)).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    rows = lib().ym_conv_fwd_stat_rows(ctypes.byref(d))
    fused = lib().ym_conv_fwd_bn_fused(ctypes.byref(d))
    assert fused == (0 if cin == 64 and h == 80 else 1)

    def run(fold):
        z = torch.empty(n, h, w, cout, dtype=torch.float16, device=dev)
        ss = torch.empty(rows, cout, device=dev)
        sq = torch.empty(rows, cout, device=dev)
        rm, rv = torch.zeros(cout, device=dev), torch.ones(cout, device=dev)
        nbt = torch.zeros(1, dtype=torch.int64, device=dev)
        out = torch.empty(4, cout, device=dev)
        ws = torch.zeros(lib().ym_bn_workspace_size(cout), dtype=torch.uint8, device=dev)
        for _ in range(3):
            if fold:
                f = BnFold(gamma=gamma.data_ptr(), beta=beta.data_ptr(), running_mean=rm.data_ptr(),
                           running_var=rv.data_ptr(), num_batches_tracked=nbt.data_ptr(), scale=out[0].data_ptr(),
                           shift=out[1].data_ptr(), mean=out[2].data_ptr(), rstd=out[3].data_ptr(),
                           workspace=ws.data_ptr(), count=float(n * h * w), momentum=0.03, eps=1e-3)
                call("ym_conv_fwd_bn", ctypes.byref(d), x.data_ptr(), wt.data_ptr(), z.data_ptr(), ss.data_ptr(),
                     sq.data_ptr(), ctypes.byref(f), st)
            else:
                call("ym_conv_fwd", ctypes.byref(d), x.data_ptr(), wt.data_ptr(), z.data_ptr(), None, ss.data_ptr(),
                     sq.data_ptr(), st)
                call("ym_bn_finalize", ss.data_ptr(), sq.data_ptr(), rows, cout, float(n * h * w), gamma.data_ptr(),
                     beta.data_ptr(), rm.data_ptr(), rv.data_ptr(), nbt.data_ptr(), 0.03, 1e-3, out[0].data_ptr(),
                     out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(), ws.data_ptr(), st)
        torch.cuda.synchronize()
        return z, out, rm, rv, nbt, ws
    z0, o0, rm0, rv0, n0, _ = run(False)
    z1, o1, rm1, rv1, n1, ws1 = run(True)
    assert torch.equal(z0, z1)
    for a, b in ((o0, o1), (rm0, rm1), (rv0, rv1)):
        assert float(((a - b).abs() / b.abs().clamp_min(1e-3)).max()) < 1e-6
    assert int(n0) == int(n1) == 3
    assert int(ws1[:256].view(torch.int32).abs().sum()) == 0          # every ticket re-armed
