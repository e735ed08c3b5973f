"""The CPU oracle is pinned against fixtures produced by running the reference
(tests/golden/gen_golden.py).  Everything here runs on CPU."""
import json

import numpy as np
import pytest
import torch

from oracle import model as om
from oracle import loss as ol
from oracle import post as op
from conftest import GOLDEN


def _batch(d):
    return {"cls": torch.from_numpy(d["cls"]), "bboxes": torch.from_numpy(d["bboxes"]),
            "batch_idx": torch.from_numpy(d["batch_idx"])}


@pytest.mark.parametrize("scale", ["n", "s", "m"])
def test_structure_keys(scale):
    ref = json.loads((GOLDEN / "structure.json").read_text())[scale]
    layers, save, P = om.build(om.load_cfg(scale))
    assert save == ref["save"]
    assert [[k, list(v.shape)] for k, v in P.items()] == [[k, s] for k, s, _ in ref["keys"]]
    n_params = sum(v.numel() for k, v in P.items() if "running" not in k and "num_batches" not in k)
    assert n_params == ref["n_params"]
    assert float(P["model.0.bn.running_var"][0]) == pytest.approx(ref["bn_running_var"])
    assert float(P["model.23.cv3.0.2.bias"][0]) == pytest.approx(ref["detect_bias_cls"])


def test_nms_oracle_bitexact(golden):
    d = golden("nms.npz")
    for n in (0, 1, 2, 100, 1000, 6700):
        keep = op.nms(d[f"n{n}_boxes"], d[f"n{n}_scores"], 0.45)
        np.testing.assert_array_equal(keep, d[f"n{n}_keep"])
    out = op.iou_row(d["iou_b1"], d["iou_b2"])
    np.testing.assert_array_equal(out.view(np.uint32), d["iou_out"].astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("kind", ["am", "lit"])
def test_decode_oracle(golden, kind):
    d = golden("decode.npz")
    outs = op.decode(d[f"{kind}_in"], 640, 0.25, 0.45)
    counts = np.asarray([len(o[1]) for o in outs])
    np.testing.assert_array_equal(counts, d[f"{kind}_counts"])
    np.testing.assert_array_equal(np.concatenate([o[0] for o in outs]), d[f"{kind}_boxes"])
    np.testing.assert_array_equal(np.concatenate([o[1] for o in outs]), d[f"{kind}_scores"])
    np.testing.assert_array_equal(np.concatenate([o[2] for o in outs]), d[f"{kind}_labels"])


def test_model_n320_forward_loss_grads(golden):
    d = golden("model_n320.npz")
    layers, save, P = om.build(om.load_cfg("n"))
    params = {k: v.requires_grad_(True) for k, v in P.items() if v.is_floating_point() and "running" not in k}
    x = torch.from_numpy(d["img"])
    heads = om.forward(P, layers, save, x, training=True)
    for i in range(3):
        torch.testing.assert_close(heads[i], torch.from_numpy(d[f"head{i}"]), rtol=1e-4, atol=1e-4)
    loss, items = ol.v8_loss(heads, _batch(d))
    torch.testing.assert_close(loss.detach().reshape(1), torch.from_numpy(d["loss"]), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(items, torch.from_numpy(d["items"]), rtol=1e-5, atol=1e-5)
    loss.backward()
    names = list(d["grad_names"])
    ref_norm = dict(zip(names, d["grad_norm"]))
    for k, p in params.items():
        if k.endswith("dfl.conv.weight"):
            continue
        r = ref_norm[k]
        assert abs(float(p.grad.norm()) - r) <= 1e-3 * max(r, 1e-3), k
    for k in [n for n in d.files if n.startswith("grad:")]:
        torch.testing.assert_close(params[k[5:]].grad, torch.from_numpy(d[k]), rtol=1e-3, atol=1e-5)
    for k in [n for n in d.files if n.startswith("state:")]:
        torch.testing.assert_close(P[k[6:]], torch.from_numpy(d[k]), rtol=1e-4, atol=1e-6)
    with torch.no_grad():
        y, feats = om.forward(P, layers, save, x, training=False)
        torch.testing.assert_close(y, torch.from_numpy(d["eval_y"]), rtol=1e-4, atol=1e-3)
        vl, vi = ol.v8_loss(feats, _batch(d))
        torch.testing.assert_close(vi, torch.from_numpy(d["eval_items"]), rtol=1e-4, atol=1e-5)


def test_assigner_and_loss_oracle(golden):
    d = golden("assigner.npz")
    feats = [torch.from_numpy(d[f"feat{i}"]).clone().requires_grad_(True) for i in range(3)]
    loss, items, inner = ol.v8_loss(feats, _batch(d), return_internals=True)
    np.testing.assert_array_equal(inner["fg"].numpy(), d["fg"])
    np.testing.assert_array_equal(inner["tgi"].numpy(), d["tgi"])
    torch.testing.assert_close(inner["target_scores"], torch.from_numpy(d["target_scores"]), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(items, torch.from_numpy(d["items"]), rtol=1e-5, atol=1e-6)
    loss.backward()
    for i in range(3):
        torch.testing.assert_close(feats[i].grad, torch.from_numpy(d[f"dfeat{i}"]), rtol=1e-4, atol=1e-6)
    # empty batch (M = 0)
    fe = [torch.from_numpy(d[f"feat{i}"]).clone().requires_grad_(True) for i in range(3)]
    empty = {"cls": torch.zeros(0, 1, dtype=torch.long), "bboxes": torch.zeros(0, 4),
             "batch_idx": torch.zeros(0, dtype=torch.long)}
    le, ie = ol.v8_loss(fe, empty)
    torch.testing.assert_close(ie, torch.from_numpy(d["empty_items"]), rtol=1e-5, atol=1e-6)
    le.backward()
    for i in range(3):
        torch.testing.assert_close(fe[i].grad, torch.from_numpy(d[f"empty_dfeat{i}"]), rtol=1e-5, atol=1e-7)


def test_precision_model_restores_and_rounds():
    """oracle/precision.py: rounding applies only inside the context and stays close to fp32."""
    from oracle.precision import hip_storage_rounding
    layers, save, P = om.build(om.load_cfg("n"))
    x = torch.rand(2, 1, 160, 160, generator=torch.Generator().manual_seed(0))
    conv0 = om.conv
    with torch.no_grad():
        ref = om.forward({k: v.clone() for k, v in P.items()}, layers, save, x, training=True)
        with hip_storage_rounding():
            assert om.conv is not conv0
            emu = om.forward({k: v.clone() for k, v in P.items()}, layers, save, x, training=True)
    assert om.conv is conv0
    for r, e in zip(ref, emu):
        err = float((r - e).norm() / r.norm())
        assert 0 < err < 2e-2


def test_oracle_training_curve_first_steps(golden):
    """The oracle's train loop (AdamW, clip 10) reproduces the reference's curve (curve.npz)."""
    from datasets.synthetic import synth_batch
    d = golden("curve.npz")
    layers, save, P = om.build(om.load_cfg("n"))
    params = [v.requires_grad_(True) for k, v in P.items()
              if v.is_floating_point() and "running" not in k and not k.endswith("dfl.conv.weight")]
    opt = torch.optim.AdamW(params, lr=1e-3, weight_decay=5e-4)
    for step in range(3):
        b = synth_batch(4, 320, seed=100 + step)
        np.testing.assert_allclose([b["img"].double().sum(), b["bboxes"].double().sum(), len(b["cls"])],
                                   d["batch_sums"][step], rtol=1e-9)
        opt.zero_grad(set_to_none=True)
        loss, items = ol.v8_loss(om.forward(P, layers, save, b["img"], training=True), b)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(params, max_norm=10.0)
        opt.step()
        np.testing.assert_allclose([float(loss), *items.tolist(), float(gn)], d["rows"][step], rtol=1e-4)


def test_metrics_oracle_matches_reference(golden):
    """oracle/metrics.py reproduces the reference's evaluate_detections on its own run."""
    from oracle import metrics as omet
    from metrics_cases import golden_case
    d = golden("metrics.npz")
    preds, tgts = golden_case(d)
    r = omet.evaluate_detections(preds, tgts, 0.25, 0.5)
    got = [r["precision"], r["recall"], r["mAP50"], r["mAP50-95"]]
    assert got == list(d["out"])


def test_metrics_oracle_ap_tie_order():
    """calculate_ap: on equal scores the TPs come first (the stable sort of tp + fp lists)."""
    from oracle import metrics as omet
    # one TP and one FP at the same score: TP first -> precision 1 at the recall step
    assert omet.calculate_ap([0.5], [0.5], 1) == pytest.approx(1.0 / (1 + 1e-6))
    assert omet.calculate_ap([], [0.9], 3) == 0.0
    assert omet.calculate_ap([0.9], [], 0) == 0.0


def _grads_vs_golden(d, P, params, rtol_norm=1e-3):
    names = list(d["grad_names"])
    ref_norm = dict(zip(names, d["grad_norm"]))
    for k, p in params.items():
        if k.endswith("dfl.conv.weight") or k not in ref_norm:
            continue
        r = ref_norm[k]
        assert abs(float(p.grad.norm()) - r) <= rtol_norm * max(r, 1e-3), (k, float(p.grad.norm()), r)
    for k in [n for n in d.files if n.startswith("grad:")]:
        torch.testing.assert_close(params[k[5:]].grad, torch.from_numpy(d[k]), rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("scale,name", [("s", "model_s128.npz"), ("m", "model_m256.npz")])
def test_model_s_m_forward_loss_grads(golden, scale, name):
    """The s (C2PSA heads=4) and m (1024-channel layers, heads=8) graphs at small resolution."""
    d = golden(name)
    layers, save, P = om.build(om.load_cfg(scale))
    params = {k: v.requires_grad_(True) for k, v in P.items() if v.is_floating_point() and "running" not in k}
    heads = om.forward(P, layers, save, torch.from_numpy(d["img"]), training=True)
    for i in range(3):
        torch.testing.assert_close(heads[i], torch.from_numpy(d[f"head{i}"]), rtol=1e-4, atol=1e-4)
    loss, items = ol.v8_loss(heads, _batch(d))
    torch.testing.assert_close(loss.detach().reshape(1), torch.from_numpy(d["loss"]), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(items, torch.from_numpy(d["items"]), rtol=1e-5, atol=1e-5)
    loss.backward()
    if "grad_names" not in d.files:          # model_s128: norms in parameter order
        names = [k for k in P if P[k].is_floating_point() and "running" not in k]
        ref = dict(zip(names, d["grad_norm"]))
        for k, p in params.items():
            if not k.endswith("dfl.conv.weight"):
                assert abs(float(p.grad.norm()) - ref[k]) <= 1e-3 * max(ref[k], 1e-3), k
        for k in [n for n in d.files if n.startswith("grad:")]:
            torch.testing.assert_close(params[k[5:]].grad, torch.from_numpy(d[k]), rtol=1e-3, atol=1e-5)
    else:
        _grads_vs_golden(d, P, params)


def attn_big_case(name):
    """(P, x, dy) of the attn_big.npz cases: C2PSA(c, c, 1) with key-seeded weights."""
    c, shape, seed = {"h4n400": (512, (2, 512, 20, 20), 51), "h8n1600": (1024, (1, 1024, 40, 40), 52)}[name]
    P = om.block_params({"type": "C2PSA", "c1": c, "c2": c, "n": 1})
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(shape, generator=g)
    dy = torch.randn(shape, generator=g)
    return P, x, dy


def fingerprint(t, n=16384):
    flat = t.detach().reshape(-1)
    step = max(1, flat.numel() // n)
    return flat[::step][:n]


@pytest.mark.parametrize("name", ["h4n400", "h8n1600"])
def test_c2psa_big_heads_oracle(golden, name):
    """C2PSA at the s@640 (heads 4, N 400) and m@1280 (heads 8, N 1600) attention shapes."""
    d = golden("attn_big.npz")
    P, x, dy = attn_big_case(name)
    params = {k: v.requires_grad_(True) for k, v in P.items() if v.is_floating_point() and "running" not in k}
    x.requires_grad_(True)
    y = om.c2psa(P, "blk", x, 1)
    y.backward(dy)
    torch.testing.assert_close(fingerprint(y), torch.from_numpy(d[f"{name}/y_fp"]), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(fingerprint(x.grad), torch.from_numpy(d[f"{name}/dx_fp"]), rtol=1e-4, atol=1e-4)
    ref = dict(zip(d[f"{name}/grad_names"], d[f"{name}/grad_norm"]))
    for k, v in ref.items():
        assert abs(float(params["blk." + k].grad.norm()) - v) <= 1e-3 * max(v, 1e-3), k
    torch.testing.assert_close(fingerprint(params["blk.m.0.attn.qkv.conv.weight"].grad),
                               torch.from_numpy(d[f"{name}/qkv_grad_fp"]), rtol=1e-3, atol=1e-5)


def test_detect_standalone_oracle(golden):
    """oracle.model.detect against the reference's Detect called on its own (detect.npz)."""
    d = golden("detect.npz")
    P = {"d." + k[2:]: torch.from_numpy(d[k]).clone() for k in d.files if k.startswith("p:")}
    params = {k: v.requires_grad_(True) for k, v in P.items()
              if v.is_floating_point() and "running" not in k and "dfl" not in k}
    xs = [torch.from_numpy(d[f"x{i}"]).clone().requires_grad_(True) for i in range(3)]
    ys = om.detect(P, "d", xs, 5, (8.0, 16.0, 32.0), tr=True)
    for i in range(3):
        torch.testing.assert_close(ys[i], torch.from_numpy(d[f"y{i}"]), rtol=1e-4, atol=1e-4)
    torch.autograd.backward(ys, [torch.from_numpy(d[f"dy{i}"]) for i in range(3)])
    for i in range(3):
        torch.testing.assert_close(xs[i].grad, torch.from_numpy(d[f"dx{i}"]), rtol=1e-4, atol=1e-4)
    for k, p in params.items():
        torch.testing.assert_close(p.grad, torch.from_numpy(d["g:" + k[2:]]), rtol=1e-3, atol=1e-4)
    for k in [n for n in d.files if n.startswith("s:")]:
        torch.testing.assert_close(P["d." + k[2:]], torch.from_numpy(d[k]), rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        y, maps = om.detect(P, "d", [x.detach() for x in xs], 5, (8.0, 16.0, 32.0), tr=False)
    torch.testing.assert_close(y, torch.from_numpy(d["eval_y"]), rtol=1e-4, atol=1e-3)
