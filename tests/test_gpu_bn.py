"""The one-launch BatchNorm finalize (bn.hip bn_finalize_fused_kernel) on its own, against a host fp64
reduction of the same partial rows.

The kernel folds [G][C] partial rows in one launch: (C/64) x 32 level-1 workgroups publish fp64 rows with
write-through stores, take a ticket, and the last arriver of each channel group folds the 32 rows and
writes the finalize (forward: scale / shift / mean / rstd and the running statistics of BatchNorm2d,
models/yolo11_modules.py:29 with eps 1e-3 / momentum 0.03 from yolo11_model.py:183-185; backward: dgamma,
dbeta and the apply coefficients).  The hand-off rests on relaxed agent-scope atomics (bn.hip header), so
this drives it with many workgroups (up to 8 x 32 = 256), back-to-back launches on one workspace (the
tickets must re-arm), and checks every channel.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("G,C", [(4096, 512), (1024, 64), (37, 200), (2048, 2048)])
def test_bn_finalize_vs_host_fp64(G, C):
    from yolomi._lib import call, lib, stream_ptr
    dev = torch.device("cuda", 0)
    st = stream_ptr(dev)
    ws = torch.zeros((lib().ym_bn_workspace_size(C) + 3) // 4, dtype=torch.float32, device=dev)
    g = torch.Generator().manual_seed(G + C)
    count = float(G * 97)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    rm0, rv0 = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    gd, bd = gamma.to(dev), beta.to(dev)
    rm, rv = rm0.clone().to(dev), rv0.clone().to(dev)
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    out = torch.empty(4, C, device=dev)
    exp_rm, exp_rv = rm0.double(), rv0.double()
    for rep in range(3):                       # back to back on one workspace: tickets re-arm
        mu_true = torch.randn(C, generator=g) * 3
        ps = (torch.randn(G, C, generator=g) + mu_true) * 97.0          # per-row sums of 97 pixels
        pq = (torch.rand(G, C, generator=g) * 5 + mu_true ** 2 + 1) * 97.0
        psd, pqd = ps.to(dev), pq.to(dev)       # kept alive: a temporary's block is reused at once
        call("ym_bn_finalize", psd.data_ptr(), pqd.data_ptr(), G, C, count, gd.data_ptr(),
             bd.data_ptr(), rm.data_ptr(), rv.data_ptr(), nbt.data_ptr(), 0.03, 1e-3, out[0].data_ptr(),
             out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(), ws.data_ptr(), st)
        torch.cuda.synchronize()
        s, q = ps.double().sum(0), pq.double().sum(0)
        mean = s / count
        var = (q / count - mean * mean).clamp_min(0)
        rstd = 1.0 / torch.sqrt(var + 1e-3)
        sc = gamma.double() * rstd
        exp_rm = 0.97 * exp_rm + 0.03 * mean
        exp_rv = 0.97 * exp_rv + 0.03 * var * count / (count - 1)
        got = out.double().cpu()
        np.testing.assert_allclose(got[0], sc, rtol=1e-6)
        np.testing.assert_allclose(got[1], beta.double() - mean * sc.float().double(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(got[2], mean, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(got[3], rstd, rtol=1e-6)
        np.testing.assert_allclose(rm.double().cpu(), exp_rm, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(rv.double().cpu(), exp_rv, rtol=1e-5)
        assert int(nbt) == rep + 1
    assert int((ws[:64].view(torch.int32) != 0).sum()) == 0      # ticket counters left at zero


@pytest.mark.parametrize("G,C", [(512, 256), (3000, 128)])
def test_bn_bwd_finalize_vs_host_fp64(G, C):
    from yolomi._lib import call, lib, stream_ptr
    dev = torch.device("cuda", 0)
    st = stream_ptr(dev)
    ws = torch.zeros((lib().ym_bn_workspace_size(C) + 3) // 4, dtype=torch.float32, device=dev)
    g = torch.Generator().manual_seed(G * 3 + C)
    count = float(G * 50)
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    rstd = (torch.rand(C, generator=g) + 0.2).to(dev)
    for rep in range(2):
        ps, pd = torch.randn(G, C, generator=g), torch.randn(G, C, generator=g)
        dgam = torch.full((C,), 0.5, device=dev)
        dbet = torch.full((C,), -0.25, device=dev)
        coef = torch.empty(3, C, device=dev)
        psd, pdd = ps.to(dev), pd.to(dev)
        call("ym_bn_bwd_finalize", psd.data_ptr(), pdd.data_ptr(), G, C, count, gamma.data_ptr(),
             rstd.data_ptr(), dgam.data_ptr(), dbet.data_ptr(), rep, coef.data_ptr(), ws.data_ptr(), st)
        torch.cuda.synchronize()
        s, q = ps.double().sum(0), pd.double().sum(0)
        np.testing.assert_allclose(dbet.double().cpu(), s + (-0.25 if rep else 0.0), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(dgam.double().cpu(), q + (0.5 if rep else 0.0), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(coef[0].double().cpu(), (gamma * rstd).double().cpu(), rtol=1e-6)
        np.testing.assert_allclose(coef[1].double().cpu(), s / count, rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(coef[2].double().cpu(), q / count, rtol=1e-5, atol=1e-9)


# ym_bn_bwd_reduce_fold: the backward statistics and finalize in one launch on the small maps (the last workgroup of
# each 64-channel group folds its rows) against the two launches it replaces: dgamma / dbeta (overwrite, then
# accumulate) and the apply coefficients to 1e-6, three calls in a row (tickets re-armed), SiLU on and off,
# a channel-slice view of dy; a map past the size limit falls back to the two launches.
@pytest.mark.parametrize("m,c,act,extra", [(25600, 128, 1, 0), (400 * 7, 512, 1, 64), (102400, 64, 0, 0),
                                           (200000, 128, 1, 0), (25600, 256, 0, 0), (25600, 256, 1, 256),
                                           (25600, 64, 0, 64), (25600, 512, 0, 0)])
def test_bn_bwd_reduce_fold_matches_two_launches(m, c, act, extra):
    import ctypes
    from yolomi._lib import call, lib
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(c + m)
    hw = 400 if m % 400 == 0 else m
    z = torch.randn(m, c, generator=g).half().to(dev)
    dyb = torch.zeros(m, c + extra, dtype=torch.bfloat16, device=dev)
    dyb[:, :c] = torch.randn(m, c, generator=g).bfloat16().to(dev)
    scale = (1 + 0.1 * torch.randn(c, generator=g)).to(dev)
    shift = (0.1 * torch.randn(c, generator=g)).to(dev)
    mean = (0.05 * torch.randn(c, generator=g)).to(dev)
    rstd = (1 + 0.1 * torch.rand(c, generator=g)).to(dev)
    gamma = (1 + 0.1 * torch.randn(c, generator=g)).to(dev)
    Gb = lib().ym_bn_bwd_blocks(m, c)
    assert lib().ym_bn_bwd_fold_ok(m, c) == (1 if m <= 25600 else 0)
    st = torch.cuda.current_stream().cuda_stream
    d_bs, d_ld = hw * (c + extra), c + extra

    def run(fused):
        ps, pg = torch.empty(Gb, c, device=dev), torch.empty(Gb, c, device=dev)
        dg, db = torch.zeros(c, device=dev), torch.zeros(c, device=dev)
        coef = torch.empty(3, c, device=dev)
        ws = torch.zeros(lib().ym_bn_workspace_size(c), dtype=torch.uint8, device=dev)
        outs = []
        for acc in (0, 1, 1):
            if fused:
                call("ym_bn_bwd_reduce_fold", dyb.data_ptr(), d_bs, d_ld, z.data_ptr(), m, c, hw, scale.data_ptr(),
                     shift.data_ptr(), mean.data_ptr(), rstd.data_ptr(), act, ps.data_ptr(), pg.data_ptr(),
                     gamma.data_ptr(), dg.data_ptr(), db.data_ptr(), acc, coef.data_ptr(), ws.data_ptr(), st)
            else:
                call("ym_bn_bwd_reduce", dyb.data_ptr(), d_bs, d_ld, z.data_ptr(), m, c, hw, scale.data_ptr(),
                     shift.data_ptr(), mean.data_ptr(), rstd.data_ptr(), act, ps.data_ptr(), pg.data_ptr(), st)
                call("ym_bn_bwd_finalize", ps.data_ptr(), pg.data_ptr(), Gb, c, float(m), gamma.data_ptr(),
                     rstd.data_ptr(), dg.data_ptr(), db.data_ptr(), acc, coef.data_ptr(), ws.data_ptr(), st)
            torch.cuda.synchronize()
            outs.append((dg.clone(), db.clone(), coef.clone()))
        assert int(ws[:256].view(torch.int32).abs().sum()) == 0
        return outs
    ref, got = run(False), run(True)
    for (a1, b1, c1), (a2, b2, c2) in zip(ref, got):
        for x, y in ((a1, a2), (b1, b2), (c1, c2)):
            # different fp32 partial groupings of the same sums: relative to the sum's magnitude (a channel's
            # sum can cancel to ~0, so the floor is 1 % of the largest channel's)
            err = float(((x - y).abs() / (y.abs() + 1e-2 * y.abs().max())).max())
            assert err < 1e-4, err
