"""BatchNorm statistics finalized inside the producing kernel (bnfold.h) vs the separate finalize
launches, on every producer: the pipelined, halo and 2-stage conv forwards (ym_conv_fwd_bn), the stem
conv (ym_conv_first_fwd_bn), the depthwise conv (ym_dw3x3_fwd_bn) and the backward statistics pass
(ym_bn_bwd_reduce_finalize).

Both paths sum the same fp32 partial rows in fp64, in different fixed orders, so the outputs agree
to ~1e-6 relative (tolerance 1e-5); each fused path is bit-identical across repeated launches (its
ticket counters re-arm themselves) and increments num_batches_tracked once per launch."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _desc(n, h, w, cin, cout, k, s):
    from yolomi._lib import ConvDesc
    p = k // 2
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    d = ConvDesc()
    d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, oh, ow, cout, k, s, p
    d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * cin, cin, oh * ow * cout, cout
    d.out_f32, d.accumulate = 2, 0
    return d, oh, ow


class _BN:
    def __init__(self, c, dev, g):
        from yolomi._lib import lib
        self.c = c
        self.gamma = (1 + 0.1 * torch.randn(c, generator=g)).to(dev)
        self.beta = (0.1 * torch.randn(c, generator=g)).to(dev)
        self.rm0 = (0.1 * torch.randn(c, generator=g)).to(dev)
        self.rv0 = (1 + 0.1 * torch.rand(c, generator=g)).to(dev)
        self.ws = torch.zeros(lib().ym_bn_workspace_size(c) // 4 + 1, dtype=torch.float32, device=dev)

    def fresh(self):
        d = self.gamma.device
        o = {k: torch.full((self.c,), float("nan"), device=d) for k in ("scale", "shift", "mean", "rstd")}
        o["rm"], o["rv"] = self.rm0.clone(), self.rv0.clone()
        o["nbt"] = torch.zeros(1, dtype=torch.int64, device=d)
        return o

    def train(self, o):
        from yolomi._lib import BnTrain
        t = BnTrain()
        t.gamma, t.beta = self.gamma.data_ptr(), self.beta.data_ptr()
        t.running_mean, t.running_var, t.num_batches_tracked = o["rm"].data_ptr(), o["rv"].data_ptr(), o["nbt"].data_ptr()
        t.momentum, t.eps = 0.03, 1e-3
        t.scale, t.shift, t.mean, t.rstd = (o[k].data_ptr() for k in ("scale", "shift", "mean", "rstd"))
        t.workspace = self.ws.data_ptr()
        return t

    def finalize(self, o, ss, sq, rows, count, st):
        from yolomi._lib import call
        call("ym_bn_finalize", ss.data_ptr(), sq.data_ptr(), rows, self.c, float(count), self.gamma.data_ptr(),
             self.beta.data_ptr(), o["rm"].data_ptr(), o["rv"].data_ptr(), o["nbt"].data_ptr(), 0.03, 1e-3,
             o["scale"].data_ptr(), o["shift"].data_ptr(), o["mean"].data_ptr(), o["rstd"].data_ptr(),
             self.ws.data_ptr(), st)


def _close(a, b, tol=1e-5):
    for k in ("scale", "shift", "mean", "rstd", "rm", "rv"):
        x, y = a[k].double().cpu(), b[k].double().cpu()
        assert torch.isfinite(x).all(), k
        err = float((x - y).abs().max() / y.abs().max().clamp_min(1e-12))
        assert err < tol, (k, err)
    assert int(a["nbt"]) == 1 and int(b["nbt"]) == 1


def _same(a, b):
    for k in ("scale", "shift", "mean", "rstd", "rm", "rv"):
        assert torch.equal(a[k], b[k]), k


CONVS = [  # shape, pipe policy: (n, h, w, cin, cout, k, s)
    ((16, 64, 64, 128, 128, 3, 1), 2, 2),     # pipelined kernel, 256x128 tiles
    ((12, 80, 80, 64, 64, 3, 1), 2, 2),       # pipelined kernel, 256x64 tiles
    ((5, 20, 20, 96, 64, 3, 1), 0, 1),        # halo kernel (map <= 24 wide)
    ((2, 13, 13, 128, 136, 3, 2), 0, 0),      # 2-stage implicit GEMM, 2 channel tiles
    ((3, 9, 7, 520, 264, 1, 1), 0, 0),
]


@pytest.mark.parametrize("case", CONVS, ids=[f"n{c[0][0]}h{c[0][1]}c{c[0][3]}o{c[0][4]}k{c[0][5]}s{c[0][6]}"
                                             for c in CONVS])
def test_conv_fwd_bn_matches_separate_finalize(case):
    from yolomi._lib import call, lib
    shape, pipe, algo = case
    n, h, w, cin, cout, k, s = shape
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(11)
    d, oh, ow = _desc(*shape)
    x = (torch.randn(n, h, w, cin, generator=g) + 0.3).half().to(dev)
    wf = (torch.randn(cout, k, k, cin, generator=g) * (2.0 / (cin * k * k)) ** 0.5).half().to(dev)
    bn = _BN(cout, dev, g)
    prev = lib().ym_conv_set_pipe(pipe)
    try:
        assert lib().ym_conv_algo(ctypes.byref(d), 0) == algo
        rows = lib().ym_conv_fwd_stat_rows(ctypes.byref(d))
        st = torch.cuda.current_stream().cuda_stream
        M = n * oh * ow
        ss = torch.empty(rows, cout, device=dev)
        sq = torch.empty(rows, cout, device=dev)
        z0 = torch.empty(M, cout, dtype=torch.float16, device=dev)
        call("ym_conv_fwd", ctypes.byref(d), x.data_ptr(), wf.data_ptr(), z0.data_ptr(), None, ss.data_ptr(),
             sq.data_ptr(), st)
        ref = bn.fresh()
        bn.finalize(ref, ss, sq, rows, M, st)
        outs = []
        for _ in range(3):
            o = bn.fresh()
            t = bn.train(o)
            z1 = torch.empty_like(z0)
            call("ym_conv_fwd_bn", ctypes.byref(d), x.data_ptr(), wf.data_ptr(), z1.data_ptr(), ss.data_ptr(),
                 sq.data_ptr(), ctypes.byref(t), st)
            outs.append((o, z1))
        torch.cuda.synchronize()
    finally:
        lib().ym_conv_set_pipe(prev)
    _close(outs[0][0], ref)
    assert torch.equal(outs[0][1], z0)
    for o, _ in outs[1:]:
        _same(o, outs[0][0])
    assert int(bn.ws[:64].view(torch.int32).abs().sum()) == 0          # counters re-armed


def test_stem_and_dw_fwd_bn_match_separate_finalize():
    from yolomi._lib import call
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    st = torch.cuda.current_stream().cuda_stream
    # stem: 1 -> 32 channels, 3x3 stride 2 on a 2 x 96 x 80 image
    n, H, W, co = 2, 96, 80, 32
    oh, ow = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    img = torch.rand(n, H, W, generator=g).to(dev)
    w = (torch.randn(co, 1, 3, 3, generator=g) * 0.3).to(dev)
    bn = _BN(co, dev, g)
    blocks, M = 64, n * oh * ow
    ss, sq = torch.empty(blocks, co, device=dev), torch.empty(blocks, co, device=dev)
    z0 = torch.empty(M, co, dtype=torch.float16, device=dev)
    call("ym_conv_first_fwd", img.data_ptr(), w.data_ptr(), z0.data_ptr(), ss.data_ptr(), sq.data_ptr(), n, H, W, oh,
         ow, co, 2, 1, blocks, st)
    ref = bn.fresh()
    bn.finalize(ref, ss, sq, blocks, M, st)
    o = bn.fresh()
    t = bn.train(o)
    z1 = torch.empty_like(z0)
    call("ym_conv_first_fwd_bn", img.data_ptr(), w.data_ptr(), z1.data_ptr(), ss.data_ptr(), sq.data_ptr(), n, H, W,
         oh, ow, co, 2, 1, blocks, ctypes.byref(t), st)
    torch.cuda.synchronize()
    _close(o, ref)
    assert torch.equal(z0, z1)
    # depthwise 3x3 on 64 channels of a 128-channel view (gsz 32, gstride 64, goff 32: the v slices)
    n, h, wd, c = 3, 20, 20, 64
    x = torch.randn(n, h, wd, 128, generator=g).half().to(dev)
    wdw = (torch.randn(c, 9, generator=g) * 0.3).to(dev)
    bn = _BN(c, dev, g)
    blocks, M = 32, n * h * wd
    ss, sq = torch.empty(blocks, c, device=dev), torch.empty(blocks, c, device=dev)
    z0 = torch.empty(M, c, dtype=torch.float16, device=dev)
    call("ym_dw3x3_fwd", x.data_ptr(), h * wd * 128, 128, 32, 64, 32, wdw.data_ptr(), z0.data_ptr(), ss.data_ptr(),
         sq.data_ptr(), n, h, wd, c, blocks, st)
    ref = bn.fresh()
    bn.finalize(ref, ss, sq, blocks, M, st)
    o = bn.fresh()
    t = bn.train(o)
    z1 = torch.empty_like(z0)
    call("ym_dw3x3_fwd_bn", x.data_ptr(), h * wd * 128, 128, 32, 64, 32, wdw.data_ptr(), z1.data_ptr(),
         ss.data_ptr(), sq.data_ptr(), n, h, wd, c, blocks, ctypes.byref(t), st)
    torch.cuda.synchronize()
    _close(o, ref)
    assert torch.equal(z0, z1)


@pytest.mark.parametrize("m,c,act", [(64 * 80 * 80, 64, 1), (64 * 20 * 20, 512, 1), (3 * 7 * 5, 24, 0)])
def test_bwd_reduce_finalize_matches_separate(m, c, act):
    from yolomi._lib import call, lib
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(m % 1000 + c)
    st = torch.cuda.current_stream().cuda_stream
    hw = m // (64 if m % 64 == 0 else 3)
    dy = torch.randn(m, c, generator=g).bfloat16().to(dev)
    z = torch.randn(m, c, generator=g).half().to(dev)
    sc, sh = (1 + 0.1 * torch.randn(c, generator=g)).to(dev), (0.1 * torch.randn(c, generator=g)).to(dev)
    mu, rs = (0.1 * torch.randn(c, generator=g)).to(dev), (1 + 0.1 * torch.rand(c, generator=g)).to(dev)
    gamma = (1 + 0.1 * torch.randn(c, generator=g)).to(dev)
    blocks = lib().ym_bn_bwd_blocks(m, c)
    ws = torch.zeros(lib().ym_bn_workspace_size(c) // 4 + 1, dtype=torch.float32, device=dev)
    res = []
    for fused in (0, 1, 1):
        ps, pd = torch.empty(blocks, c, device=dev), torch.empty(blocks, c, device=dev)
        dgam, dbet = torch.full((c,), 0.5, device=dev), torch.full((c,), -0.5, device=dev)
        coef = torch.full((3, c), float("nan"), device=dev)
        args = (dy.data_ptr(), hw * c, c, z.data_ptr(), m, c, hw, sc.data_ptr(), sh.data_ptr(), mu.data_ptr(),
                rs.data_ptr(), act, ps.data_ptr(), pd.data_ptr())
        if fused:
            call("ym_bn_bwd_reduce_finalize", *args, gamma.data_ptr(), dgam.data_ptr(), dbet.data_ptr(), 1,
                 coef.data_ptr(), ws.data_ptr(), st)
        else:
            call("ym_bn_bwd_reduce", *args, st)
            call("ym_bn_bwd_finalize", ps.data_ptr(), pd.data_ptr(), blocks, c, float(m), gamma.data_ptr(),
                 rs.data_ptr(), dgam.data_ptr(), dbet.data_ptr(), 1, coef.data_ptr(), ws.data_ptr(), st)
        res.append((dgam, dbet, coef))
    torch.cuda.synchronize()
    for a, b in zip(res[1], res[0]):
        err = float((a.double() - b.double()).abs().max() / b.double().abs().max())
        assert torch.isfinite(a).all() and err < 1e-5, err
    for a, b in zip(res[2], res[1]):
        assert torch.equal(a, b)
    assert int(ws[:64].view(torch.int32).abs().sum()) == 0
