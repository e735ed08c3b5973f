"""GPU parity of the HIP training path against the reference goldens and the CPU oracle.

Tolerances (BASELINE.json north_star: 1e-2 for 16-bit tensors): activations are fp16 and
gradients bf16, so single blocks are held to relative-L2 <= 1e-2 (outputs) / 2e-2 (input and
parameter gradients); the full n@320 network's head maps to <= 1e-2; loss items <= 1e-2;
EVERY parameter gradient within 10%, or within 2x the distance of the oracle run under the
HIP storage-rounding model (oracle/precision.py) where that is larger: backbone gradients are
discontinuous in the activations through SPPF's max-pool routing — stated per assert.  The loss
on fp32 head maps is an fp32 path: assignment decisions (fg mask, target_gt_idx) are bit-exact
and loss values / head gradients within 1e-4.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


BLOCKS = {
    "conv3s1": lambda M: M.Conv(32, 64, 3, 1),
    "conv3s2": lambda M: M.Conv(32, 64, 3, 2),
    "conv1": lambda M: M.Conv(64, 32, 1, 1),
    "conv0": lambda M: M.Conv(1, 32, 3, 2),
    "c3k2": lambda M: M.C3k2(64, 64, 1, False, 0.25),
    "c3k2k": lambda M: M.C3k2(64, 128, 1, True),
    "sppf": lambda M: M.SPPF(128, 128, 5),
    "c2psa": lambda M: M.C2PSA(256, 256, 1),
}


@pytest.mark.parametrize("name", list(BLOCKS))
def test_block_fwd_bwd_vs_reference(golden, name):
    import models as M
    d = golden("blocks.npz")
    mod = BLOCKS[name](M)
    sd = {k[len(name) + 3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith(name + "/p:")}
    mod.load_state_dict(sd)
    for m in mod.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.eps, m.momentum = 1e-3, 0.03
    mod = mod.cuda().train()
    x = torch.from_numpy(d[name + "/x"]).cuda().requires_grad_(name != "conv0")
    y = mod(x)
    assert rel(y, d[name + "/y"]) < 1e-2, ("y", rel(y, d[name + "/y"]))
    y.backward(torch.from_numpy(d[name + "/dy"]).cuda())
    if name != "conv0":
        # max-pool gradient routing is discontinuous in its input: with bf16 activations a few
        # near-tied 5x5 windows pick a different argmax than the fp32 reference, moving whole
        # routed sums; SPPF's dx is therefore held to 1e-1 (its pool kernels are checked for
        # exactness on identical inputs in test_sppf_pool_chain_exact)
        tol = 1e-1 if name == "sppf" else 2e-2
        assert rel(x.grad, d[name + "/dx"]) < tol, ("dx", rel(x.grad, d[name + "/dx"]))
    # a BN bias whose output reaches the loss only linearly through later training-mode BNs has an
    # exactly-zero true gradient (BN removes per-channel shifts); compare those on the block's grad scale
    scale = max(float(np.linalg.norm(d[f"{name}/g:{k}"])) for k, p in mod.named_parameters() if p.requires_grad)
    for k, p in mod.named_parameters():
        if not p.requires_grad:
            continue
        ref = d[f"{name}/g:{k}"]
        err = float((p.grad.double().cpu() - torch.from_numpy(ref).double()).norm())
        tol = 1e-1 if name == "sppf" else 3e-2
        assert err < tol * max(float(np.linalg.norm(ref)), 5e-3 * scale), (k, err, float(np.linalg.norm(ref)))
    for k, v in mod.state_dict().items():
        if "running" in k:
            assert rel(v, d[f"{name}/s:{k}"]) < 1e-2, (k, rel(v, d[f"{name}/s:{k}"]))


def _batch(d, dev="cuda"):
    return {"img": torch.from_numpy(d["img"]).to(dev), "batch_idx": torch.from_numpy(d["batch_idx"]).to(dev),
            "cls": torch.from_numpy(d["cls"]).to(dev), "bboxes": torch.from_numpy(d["bboxes"]).to(dev)}


def _seeded_model(scale, nc=5, ch=1):
    from oracle import model as om
    from models import build_yolo11
    cfg = om.load_cfg(scale)
    layers, save, P = om.build(cfg, ch=ch, nc=nc)
    m = build_yolo11(cfg, ch=ch, nc=nc)
    m.load_state_dict(P)
    return m.cuda()


def test_model_n320_train_step_vs_reference(golden):
    """n@320 bs2: heads, loss / items, every parameter gradient (test_gpu_network.check_network) and
    the BN running statistics after the step, against the reference's own run."""
    from losses import v8DetectionLoss
    from test_gpu_network import check_network
    d = golden("model_n320.npz")
    m = _seeded_model("n").train()
    batch = _batch(d)
    heads = m(batch["img"])
    crit = v8DetectionLoss(m)
    loss, items = crit(heads, batch)
    ref_norm = dict(zip(list(d["grad_names"]), d["grad_norm"]))
    full = {k[5:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("grad:")}
    worst = check_network("n", heads, loss, items, m, [torch.from_numpy(d[f"head{i}"]) for i in range(3)],
                          d["loss"][0], d["items"], ref_norm, full, d["img"],
                          {k: v.cpu() for k, v in batch.items() if k != "img"})
    print("worst err/tol", worst)
    sd = m.state_dict()
    for k in [n for n in d.files if n.startswith("state:")]:
        assert rel(sd[k[6:]], d[k]) < 2e-2, (k, rel(sd[k[6:]], d[k]))


def test_assigner_and_loss_exact_fp32(golden):
    """fp32 head maps straight into the fused loss: decisions bit-exact, values/grads ~1e-5."""
    import torch.nn as nn
    from models import Detect
    from losses import v8DetectionLoss
    d = golden("assigner.npz")

    class Stub(nn.Module):
        def __init__(self):
            super().__init__()
            self.det = Detect(5, (64, 128, 256))
            self.det.stride = torch.tensor([8.0, 16.0, 32.0])
    crit = v8DetectionLoss(Stub().cuda())
    feats = [torch.from_numpy(d[f"feat{i}"]).cuda().requires_grad_(True) for i in range(3)]
    batch = {k: torch.from_numpy(d[k]).cuda() for k in ("batch_idx", "cls", "bboxes")}
    loss, items = crit(feats, batch)
    tgi, fg, nm = crit.assignment()
    np.testing.assert_array_equal(fg.cpu().numpy().astype(bool), d["fg"])
    np.testing.assert_array_equal(tgi.cpu().numpy(), d["tgi"])
    ts = torch.from_numpy(d["target_scores"])
    torch.testing.assert_close(nm.cpu() * fg.cpu(), ts.sum(-1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(items.cpu(), torch.from_numpy(d["items"]), rtol=1e-4, atol=1e-6)
    loss.backward()
    for i in range(3):
        torch.testing.assert_close(feats[i].grad.cpu(), torch.from_numpy(d[f"dfeat{i}"]), rtol=1e-3, atol=1e-6)
    # M = 0 batch
    fe = [torch.from_numpy(d[f"feat{i}"]).cuda().requires_grad_(True) for i in range(3)]
    empty = {"batch_idx": torch.zeros(0, dtype=torch.long).cuda(), "cls": torch.zeros(0, 1, dtype=torch.long).cuda(),
             "bboxes": torch.zeros(0, 4).cuda()}
    le, ie = crit(fe, empty)
    torch.testing.assert_close(ie.cpu(), torch.from_numpy(d["empty_items"]), rtol=1e-5, atol=1e-6)
    le.backward()
    for i in range(3):
        torch.testing.assert_close(fe[i].grad.cpu(), torch.from_numpy(d[f"empty_dfeat{i}"]), rtol=1e-4, atol=1e-7)


def test_model_eval_decode_vs_reference(golden):
    from losses import v8DetectionLoss
    d = golden("model_n320.npz")
    m = _seeded_model("n").train()
    batch = _batch(d)
    crit = v8DetectionLoss(m)
    loss, _ = crit(m(batch["img"]), batch)      # one train forward (BN running stats update)
    loss.backward()
    m.eval()
    # 1e-2, or 1.2x the error of the oracle under the HIP storage-rounding model (the same train
    # step, then the eval forward on the updated running statistics) where that is larger: the eval
    # y carries the DFL projection with random weights (Q5), which amplifies head-map rounding
    from oracle import model as om
    from oracle import loss as ol
    from oracle.precision import hip_storage_rounding
    layers, save, P = om.build(om.load_cfg("n"))
    img = torch.from_numpy(d["img"])
    with hip_storage_rounding():
        P = {k: (v.requires_grad_(True) if v.is_floating_point() and "running" not in k else v) for k, v in P.items()}
        ol.v8_loss(om.forward(P, layers, save, img, training=True),
                   {k: v.cpu() for k, v in batch.items() if k != "img"})[0].backward()
        with torch.no_grad():
            emu_y, emu_f = om.forward(P, layers, save, img, training=False)
            emu_vi = ol.v8_loss(emu_f, {k: v.cpu() for k, v in batch.items() if k != "img"})[1]
    with torch.no_grad():
        y, feats = m(batch["img"])
        bound = max(1e-2, 1.2 * rel(emu_y, d["eval_y"]))
        assert rel(y, d["eval_y"]) < bound, (rel(y, d["eval_y"]), bound)
        vl, vi = crit((y, feats), batch)
        bound = max(1e-2, 1.2 * rel(emu_vi, d["eval_items"]))
        assert rel(vi, d["eval_items"]) < bound, (rel(vi, d["eval_items"]), bound)


@pytest.mark.parametrize("H,W,C", [(9, 7, 16), (20, 20, 12), (48, 44, 8)])
def test_sppf_pool_chain_exact(H, W, C):
    """The three chained 5x5 pools (fwd values and first-max gradient routing) are exact on
    identical fp32 inputs, against torch CPU max_pool2d autograd (reference semantics).
    Shapes: LDS kernels with 8- and 4-channel blocks, and the direct kernels (map too big)."""
    from yolomi._lib import call, stream_ptr
    g = torch.Generator().manual_seed(0)
    B = 2
    # quantised values create exact ties like chained pools do
    x = torch.randint(-8, 8, (B, H, W, C), generator=g).float() / 4
    dys = [torch.randn(B, H, W, C, generator=g) for _ in range(3)]
    P = torch.zeros(4, B * H * W, C, device="cuda")
    P[0] = x.reshape(-1, C).cuda()
    code = torch.zeros(3, B * H * W, C, dtype=torch.uint8, device="cuda")
    yv = torch.zeros(B, H, W, C, dtype=torch.float16, device="cuda")
    st = stream_ptr()
    for j in range(3):
        call("ym_maxpool5_f32_fwd", P[j].data_ptr(), P[j + 1].data_ptr(), code[j].data_ptr(), yv.data_ptr(),
             H * W * C, C, B, H, W, C, st)
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    ys, t = [], xr
    for j in range(3):
        t = torch.nn.functional.max_pool2d(t, 5, 1, 2)
        ys.append(t)
    for j in range(3):
        torch.testing.assert_close(P[j + 1].cpu().view(B, H, W, C), ys[j].detach().permute(0, 2, 3, 1), rtol=0, atol=0)
    torch.testing.assert_close(yv.float().cpu(), ys[2].detach().permute(0, 2, 3, 1), rtol=0, atol=0)
    torch.autograd.backward(ys, [dy.permute(0, 3, 1, 2) for dy in dys])
    # chain backward with the kernels: g3 -> +dy2 -> g2 -> +dy1 -> g1 -> dx (bf16 view, accumulated
    # onto a known base); the bf16 init views carry exactly representable values
    dys_b = [d.bfloat16() for d in dys]
    ref_dys = [d.float() for d in dys_b]
    xr2 = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    ys2, t = [], xr2
    for j in range(3):
        t = torch.nn.functional.max_pool2d(t, 5, 1, 2)
        ys2.append(t)
    torch.autograd.backward(ys2, [d.permute(0, 3, 1, 2) for d in ref_dys])
    cur = ref_dys[2].reshape(-1, C).cuda().contiguous()
    for j in (2, 1):
        nxt = torch.empty(B * H * W, C, device="cuda")
        init = dys_b[j - 1].cuda().contiguous()
        call("ym_maxpool5_f32_bwd", code[j].data_ptr(), cur.data_ptr(), init.data_ptr(), H * W * C, C,
             nxt.data_ptr(), None, 0, 0, 0, B, H, W, C, st)
        cur = nxt
    base = torch.full((B, H, W, C), 0.5, dtype=torch.bfloat16, device="cuda")
    call("ym_maxpool5_f32_bwd", code[0].data_ptr(), cur.data_ptr(), None, 0, 0, None, base.data_ptr(), H * W * C, C,
         1, B, H, W, C, st)
    want = (xr2.grad.permute(0, 2, 3, 1) + 0.5).bfloat16().float()
    torch.testing.assert_close(base.float().cpu(), want, rtol=1e-2, atol=1e-2)
    # routing is exact: the fp32 chain result before the final bf16 rounding
    cur_chk = ref_dys[2].reshape(-1, C).cuda().contiguous()
    for j in (2, 1, 0):
        nxt = torch.empty(B * H * W, C, device="cuda")
        init = dys_b[j - 1].cuda().contiguous() if j > 0 else None
        call("ym_maxpool5_f32_bwd", code[j].data_ptr(), cur_chk.data_ptr(), init.data_ptr() if init is not None else None,
             H * W * C, C, nxt.data_ptr(), None, 0, 0, 0, B, H, W, C, st)
        cur_chk = nxt
    torch.testing.assert_close(cur_chk.cpu().view(B, H, W, C), xr2.grad.permute(0, 2, 3, 1), rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("H,W,C,B", [(20, 20, 16, 3), (9, 7, 12, 3), (40, 40, 8, 3), (20, 20, 256, 8),
                                     (10, 10, 128, 8)])
def test_sppf_fused_chain_bit_identical(H, W, C, B):
    """ym_sppf_fwd / ym_sppf_bwd (the three pools in one launch, chain in LDS) against three chained
    ym_maxpool5_f32_fwd / _bwd launches on the same inputs: pool values, argmax codes, fp16 slices,
    the fp32 routed gradient and the accumulated bf16 slice-0 gradient all bit-identical.
    Shapes: forward blocks of 8 / 4 channels (8 images) and 2 / 1 (3 images: the small-batch grid), odd maps, the
    m@1280 40x40 map."""
    from yolomi._lib import call, lib, stream_ptr
    assert lib().ym_sppf_supported(H, W, C)
    g = torch.Generator().manual_seed(H * W + C)
    M = B * H * W
    x = (torch.randint(-8, 8, (M, C), generator=g).float() / 4).cuda()    # exact ties, as chained pools make
    st = stream_ptr()
    # reference: chained per-pool launches
    P = torch.zeros(4, M, C, device="cuda")
    P[0] = x
    code = torch.zeros(3, M, C, dtype=torch.uint8, device="cuda")
    ybuf = torch.zeros(B, H, W, 4 * C, dtype=torch.float16, device="cuda")      # concat [s0 | s1 | s2 | s3]
    bs, ld = H * W * 4 * C, 4 * C
    sl = lambda t, j: t.data_ptr() + 2 * j * C
    for j in range(3):
        call("ym_maxpool5_f32_fwd", P[j].data_ptr(), P[j + 1].data_ptr(), code[j].data_ptr(), sl(ybuf, j + 1), bs, ld,
             B, H, W, C, st)
    P2 = torch.zeros(3, M, C, device="cuda")
    code2 = torch.zeros(3, M, C, dtype=torch.uint8, device="cuda")
    ybuf2 = torch.zeros_like(ybuf)
    call("ym_sppf_fwd", x.data_ptr(), code2.data_ptr(), sl(ybuf2, 1), sl(ybuf2, 2), sl(ybuf2, 3), bs, ld,
         P2.data_ptr(), B, H, W, C, st)
    torch.cuda.synchronize()
    assert torch.equal(P[1:], P2) and torch.equal(code, code2) and torch.equal(ybuf, ybuf2)
    # backward: slice gradients in one bf16 concat gradient buffer, slice 0 accumulated onto a base
    gbuf = torch.randn(B, H, W, 4 * C, generator=g).bfloat16().cuda()
    gbuf[..., :C] = 0.25
    gref = gbuf.clone()
    cur = gbuf[..., 3 * C:].float().reshape(M, C).contiguous()
    for j in (2, 1):
        nxt = torch.empty(M, C, device="cuda")
        call("ym_maxpool5_f32_bwd", code[j].data_ptr(), cur.data_ptr(), sl(gbuf, j), bs, ld, nxt.data_ptr(), None, 0,
             0, 0, B, H, W, C, st)
        cur = nxt
    dx_ref = torch.empty(M, C, device="cuda")
    call("ym_maxpool5_f32_bwd", code[0].data_ptr(), cur.data_ptr(), None, 0, 0, dx_ref.data_ptr(), gref.data_ptr(),
         bs, ld, 1, B, H, W, C, st)
    dx32 = torch.empty(M, C, device="cuda")
    call("ym_sppf_bwd", code.data_ptr(), sl(gbuf, 1), sl(gbuf, 2), sl(gbuf, 3), bs, ld, gbuf.data_ptr(), bs, ld, 1,
         dx32.data_ptr(), B, H, W, C, st)
    torch.cuda.synchronize()
    assert torch.equal(dx32, dx_ref)
    assert torch.equal(gbuf, gref)


def _emulated_heads(scale, img, nc=5, ch=1, jitter=0):
    from oracle import model as om
    from oracle.precision import hip_storage_rounding
    layers, save, P = om.build(om.load_cfg(scale), ch=ch, nc=nc)
    with torch.no_grad(), hip_storage_rounding(jitter=jitter):
        return om.forward(P, layers, save, torch.as_tensor(img), training=True)


def _emulated_oracle_grads(scale, img, loss_fn):
    """Parameter gradients of the CPU oracle under the HIP storage-rounding model."""
    from oracle import model as om
    from oracle.precision import hip_storage_rounding
    layers, save, P = om.build(om.load_cfg(scale))
    leaf = {k: v.requires_grad_(True) for k, v in P.items()
            if v.is_floating_point() and "running" not in k and not k.endswith("dfl.conv.weight")}
    with hip_storage_rounding():
        out = om.forward(P, layers, save, torch.as_tensor(img), training=True)
        loss_fn(out).backward() if callable(loss_fn) else torch.autograd.backward(out, loss_fn)
    return {k: v.grad for k, v in leaf.items()}


def test_network_backward_fixed_head_grads_vs_oracle():
    """Network backward: the same random head gradients through our plan and through CPU fp32
    autograd of the oracle.  The backbone is discontinuous in its activations (SPPF max-pool
    routing, oracle/precision.py), so each parameter's relative-L2 error is bounded by
    max(3e-2, 2 x the error of the oracle under the HIP storage-rounding model: both round at
    the same points but differ in accumulation order, so near-tie argmax flips land elsewhere); near-zero true
    gradients are compared on the network's gradient scale."""
    from oracle import model as om
    from models import build_yolo11
    cfg = om.load_cfg("n")
    layers, save, P = om.build(cfg)
    m = build_yolo11(cfg, ch=1, nc=5)
    m.load_state_dict(P)
    m = m.cuda().train()
    g = torch.Generator().manual_seed(3)
    img = torch.rand(2, 1, 256, 256, generator=g)
    heads = m(img.cuda())
    dh = [torch.randn(h.shape, generator=g) * 0.01 for h in heads]
    torch.autograd.backward(heads, [t.cuda() for t in dh])
    Q = {k: v.clone() for k, v in P.items()}
    leaf = {k: v.requires_grad_(True) for k, v in Q.items()
            if v.is_floating_point() and "running" not in k and not k.endswith("dfl.conv.weight")}
    ref = om.forward(Q, layers, save, img, training=True)
    torch.autograd.backward(ref, dh)
    emu = _emulated_oracle_grads("n", img, dh)
    gmax = max(float(v.grad.norm()) for v in leaf.values())
    worst = []
    for k, p in m.named_parameters():
        if not p.requires_grad:
            continue
        r = leaf[k].grad
        scale = max(float(r.norm()), 1e-4 * gmax)
        err = float((p.grad.cpu().double() - r.double()).norm()) / scale
        err_emu = float((emu[k].double() - r.double()).norm()) / scale
        bound = max(3e-2, 2.0 * err_emu)
        worst.append((err / bound, k, err, err_emu))
        assert err < bound, (k, err, err_emu)
    print("worst err/bound", sorted(worst)[-3:])


def test_loss_with_host_max_gt_matches_synced_count():
    """The loss sized by the data path's host-side max_gt equals the one that syncs to count it."""
    from oracle import model as om
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets import prepare_batch
    from datasets.synthetic import synth_batch
    cfg = om.load_cfg("n")
    _, _, P = om.build(cfg)
    m = build_yolo11(cfg, ch=1, nc=5)
    m.load_state_dict(P)
    m = m.cuda().train()
    crit = v8DetectionLoss(m)
    raw = synth_batch(3, 256, seed=8)
    b1 = prepare_batch(raw, "cuda")
    assert "max_gt" in b1
    b0 = {k: v for k, v in b1.items() if k != "max_gt"}
    heads = [h.detach().clone().requires_grad_(True) for h in m(b1["img"])]
    outs = []
    for b in (b0, b1):
        hs = [h.detach().clone().requires_grad_(True) for h in heads]
        loss, items = crit(hs, b)
        loss.backward()
        outs.append((loss.detach(), items, [h.grad for h in hs]))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    for a, c in zip(outs[0][2], outs[1][2]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("c,shape", [(32, (2, 64, 64)), (32, (3, 47, 61)), (128, (2, 40, 36))])
def test_stem_block_vs_torch_fp32(c, shape):
    """The stem Conv(1, c, 3, 2) block on its own vs PyTorch fp32 (CPU) on the same input / output gradient:
    c = 32 runs the fused stored-z backward (ym_stem_bwd_wgrad_stored, BN apply inside the weight gradient;
    odd map sizes give partial 8x32 tiles), c = 128 the generic one (ym_bn_bwd_apply + ym_conv_first_wgrad).
    y within 1e-2, parameter gradients within 2e-2, running statistics within 1e-2 (relative L2)."""
    import models as M
    g = torch.Generator().manual_seed(sum(shape) + c)
    B, H, W = shape
    x = torch.rand(B, 1, H, W, generator=g)
    ref = M.Conv(1, c, 3, 2)
    torch.nn.init.normal_(ref.conv.weight, std=0.5, generator=g)
    ref.bn.eps, ref.bn.momentum = 1e-3, 0.03
    mod = M.Conv(1, c, 3, 2)
    mod.load_state_dict(ref.state_dict())
    mod.bn.eps, mod.bn.momentum = 1e-3, 0.03
    mod = mod.cuda().train()
    y = mod(x.cuda())
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(7))
    y.backward(dy.cuda())
    # fp32 reference of Conv.forward (yolo11_modules.py:32-33) with autograd on the CPU
    w = ref.conv.weight.detach().clone().requires_grad_(True)
    gm = ref.bn.weight.detach().clone().requires_grad_(True)
    bt = ref.bn.bias.detach().clone().requires_grad_(True)
    rm, rv = ref.bn.running_mean.clone(), ref.bn.running_var.clone()
    z = torch.nn.functional.conv2d(x, w, stride=2, padding=1)
    yr = torch.nn.functional.silu(torch.nn.functional.batch_norm(z, rm, rv, gm, bt, True, 0.03, 1e-3))
    yr.backward(dy)
    assert rel(y.detach(), yr.detach()) < 1e-2
    for k, r in (("conv.weight", w.grad), ("bn.weight", gm.grad), ("bn.bias", bt.grad)):
        p = dict(mod.named_parameters())[k]
        assert rel(p.grad, r) < 2e-2, (k, rel(p.grad, r))
    assert rel(mod.bn.running_mean, rm) < 1e-2 and rel(mod.bn.running_var, rv) < 1e-2


def test_sppf_block_tie_free_vs_torch_fp32():
    """SPPF (yolo11_modules.py:92-105) as a block on inputs whose 5x5 pool maxima are tie-free: every pixel of an
    image carries a distinct value of a random permutation (spacing 1/256), the same for all channels up to a
    positive gain, and cv1 (positive weights, BN beta 1: u = xhat + 1 >= -0.73, where SiLU is still increasing)
    keeps that order through SiLU — so every window's
    maximum leads the next DISTINCT value by >= 4x the fp16 rounding of the GPU path, and the 16-bit path routes
    every pooled gradient where fp32 does (copies of one source value, which the chained pools create, are exact
    ties on both paths and resolve to the same first maximum).  The margin is asserted on the fp32 reference's
    own windows.  Bounds: y within 1e-2 and dx within 2e-2 (relative L2) against PyTorch fp32 on the CPU;
    parameter gradients within max(2e-2, 2 x the 16-bit storage model's own distance), never above 5e-2 (the
    model measures 1.6 / 2.3 % on cv1's BN weight / bias here); the fixture test above keeps random inputs at
    1e-1 (near-tied windows there).
    (cv1's BN bias gradient is sum(dy_a * silu'(u)) where sum(dy_a) = 0 exactly — cv2's BN backward makes
    every concat channel's gradient zero-mean and the pools only move it — so with beta 3, where silu' is
    nearly constant, it was a cancellation residue (0.18 relative error from bf16 gradient storage);
    beta 1 spreads silu' over 0.3-1.1.)"""
    import models as M
    F = torch.nn.functional
    g = torch.Generator().manual_seed(11)
    B, C, H, W = 2, 64, 16, 16
    base = torch.stack([torch.randperm(H * W, generator=g).view(H, W).float() / (H * W) for _ in range(B)])
    x = base.view(B, 1, H, W) * (torch.rand(1, C, 1, 1, generator=g) + 0.5)
    mod = M.SPPF(C, C, 5)
    for m_ in mod.modules():
        if isinstance(m_, torch.nn.BatchNorm2d):
            m_.eps, m_.momentum = 1e-3, 0.03
    with torch.no_grad():
        mod.cv1.conv.weight.copy_(torch.rand(mod.cv1.conv.weight.shape, generator=g) + 0.1)
        mod.cv1.bn.bias.fill_(1.0)
    ref_sd = {k: v.clone() for k, v in mod.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    P = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in ref_sd.items()
         if "num_batches" not in k}

    from oracle.precision import _ConvQ, _Round

    def block(P, xin, rounded):
        def cbs(t, pre):
            if rounded:        # the HIP path's storage points (oracle/precision.py): fp16 in / z, bf16 grads
                z = _Round.apply(_ConvQ.apply(_Round.apply(t), P[pre + ".conv.weight"], 1, 1))
            else:
                z = F.conv2d(t, P[pre + ".conv.weight"])
            u = F.batch_norm(z, P[pre + ".bn.running_mean"].detach().clone(),
                             P[pre + ".bn.running_var"].detach().clone(), P[pre + ".bn.weight"], P[pre + ".bn.bias"],
                             True, 0.03, 1e-3)
            return F.silu(u)
        a = cbs(xin, "cv1")
        p1 = F.max_pool2d(a, 5, 1, 2)
        p2 = F.max_pool2d(p1, 5, 1, 2)
        p3 = F.max_pool2d(p2, 5, 1, 2)
        return cbs(torch.cat((a, p1, p2, p3), 1), "cv2"), (a, p1, p2)
    yr, pooled = block(P, xr, False)
    for t in pooled:           # margin of every window's maximum over its next distinct value
        win = F.unfold(F.pad(t.detach(), (2, 2, 2, 2), value=-1e9), 5).view(B, t.shape[1], 25, H * W)
        mx = win.max(2, keepdim=True).values
        second = torch.where(win < mx, win, torch.full_like(win, -1e9)).max(2).values
        gap = ((mx[:, :, 0] - second) / mx[:, :, 0].abs()).min()
        assert float(gap) > 4 * 2.0 ** -11, float(gap)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    # the same block under the 16-bit storage model: its parameter-gradient distance from fp32 is the floor a
    # correct 16-bit path sits at (cv1's BN gradients are 512-pixel sums of bf16-stored, pool-routed gradients)
    Pe = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in P.items()}
    block(Pe, x.clone(), True)[0].backward(dy)
    mod.load_state_dict(ref_sd)
    mod = mod.cuda().train()
    xg = x.cuda().requires_grad_(True)
    y = mod(xg)
    y.backward(dy.cuda())
    assert rel(y.detach(), yr.detach()) < 1e-2, rel(y.detach(), yr.detach())
    assert rel(xg.grad, xr.grad) < 2e-2, rel(xg.grad, xr.grad)
    # cv1's weight gradient is exactly 0 here: every input channel is the same spatial pattern up to a gain, so
    # cv1's conv only scales that pattern per output channel and its training-mode BN removes the scale; it is
    # held on the block's gradient scale instead (as the network tests do for BN-invariant parameters)
    scale = max(float(P[k].grad.norm()) for k in P if P[k].grad is not None)
    for k, p in mod.named_parameters():
        if float(P[k].grad.norm()) < 1e-4 * scale:
            assert float(p.grad.norm()) < 2e-2 * scale, (k, float(p.grad.norm()), scale)
            continue
        tol = min(5e-2, max(2e-2, 2.0 * rel(Pe[k].grad, P[k].grad)))
        assert rel(p.grad, P[k].grad) < tol, (k, rel(p.grad, P[k].grad), tol)
