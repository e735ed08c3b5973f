"""Bit-reproducibility of a training step on the GPU.

Every reduction in the HIP path runs in a fixed order (per-block partial rows summed in row order,
waves combined in wave order; no float atomics), so the same step on the same inputs gives
bit-identical heads, loss and parameter gradients — across repeated runs, one or three scheduler
streams, the weight gradients on the side stream or in line, and eager vs HIP-graph replay.  (The reference is a single-process fp32 PyTorch loop;
reproducibility is what lets tests/test_gpu_curve.py compare 20-step curves without run-to-run drift.)
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(model, crit, b):
    model.zero_grad(set_to_none=True)
    heads = model(b["img"])
    loss, items = crit(heads, b)
    loss.backward()
    torch.cuda.synchronize()
    return (heads.detach().clone() if torch.is_tensor(heads) else [h.detach().clone() for h in heads],
            loss.detach().clone(), items.detach().clone(),
            [p.grad.detach().clone() for p in model.parameters() if p.grad is not None])


def test_train_step_bit_reproducible():
    from oracle import model as om
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    cfg = om.load_cfg("n")
    _, _, P = om.build(cfg)
    m = build_yolo11(cfg, ch=1, nc=5)
    m.load_state_dict(P)
    m = m.cuda().train()
    crit = v8DetectionLoss(m)
    b = {k: v.cuda() for k, v in synth_batch(4, 320, seed=11).items()}
    # BatchNorm running statistics move every step; restore them so each step sees the same model
    bufs = {k: v.clone() for k, v in m.state_dict().items()}
    runs = []
    os.environ["YM_GRAPH"] = "0"
    for side, streams in (("1", "3"), ("1", "3"), ("0", "3"), ("1", "1")):
        os.environ["YM_SIDE_STREAM"], os.environ["YM_STREAMS"] = side, streams
        m.load_state_dict(bufs)
        runs.append(_step(m, crit, b))
    for k in ("YM_SIDE_STREAM", "YM_STREAMS"):
        os.environ.pop(k, None)
    os.environ["YM_GRAPH"] = "1"
    # HIP-graph mode on a fresh model: eager, capture, replay
    m2 = build_yolo11(cfg, ch=1, nc=5)
    m2.load_state_dict(P)
    m2 = m2.cuda().train()
    crit2 = v8DetectionLoss(m2)
    for _ in range(3):
        m2.load_state_dict(bufs)
        # a fresh image tensor each step: the replay copies it into the graph's static input
        runs.append(_step(m2, crit2, dict(b, img=b["img"].clone())))
    os.environ.pop("YM_GRAPH", None)
    ref = runs[0]
    for other in runs[1:]:
        for a, c in zip(ref[0], other[0]):
            assert torch.equal(a, c)
        assert torch.equal(ref[1], other[1]) and torch.equal(ref[2], other[2])
        for i, (a, c) in enumerate(zip(ref[3], other[3])):
            assert torch.equal(a, c), f"parameter {i}: max |diff| {float((a - c).abs().max())}"


def test_eval_coefficients_follow_replaced_buffers():
    """The eval forward computes every BatchNorm's scale / shift in one launch over a pointer table built
    once per plan (ym_bn_eval_coeff_batch).  The table is keyed on every pointer it holds, so a buffer or
    parameter REPLACED by a new tensor (bn.running_var = ..., load_state_dict(assign=True)) is read from
    its new storage, never from the freed one: the output equals a fresh model's with the same state."""
    import yaml
    from pathlib import Path
    from models import build_yolo11
    root = Path(__file__).resolve().parents[1] / "yolo-scratch_amd"
    cfg = yaml.safe_load((root / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "n"
    torch.manual_seed(3)
    m = build_yolo11(cfg, ch=1, nc=5).cuda().eval()
    img = torch.rand(2, 1, 256, 256, generator=torch.Generator().manual_seed(4)).cuda()

    def run(model):
        with torch.no_grad():
            y, _ = model(img)
        return y.clone()
    y0 = run(m)
    bn = m.model[1].bn
    bn.running_var = bn.running_var.detach().clone() * 2.0          # new storage
    bn.bias = torch.nn.Parameter(bn.bias.detach().clone() + 0.25)   # new Parameter
    y1 = run(m)
    torch.manual_seed(3)
    m2 = build_yolo11(cfg, ch=1, nc=5).cuda().eval()
    m2.load_state_dict(m.state_dict())
    y2 = run(m2)
    assert not torch.equal(y1, y0)
    assert torch.equal(y1, y2)


def test_graph_replay_gradient_accumulation():
    """gradient accumulation (two backwards without zero_grad in between) under HIP-graph
    replay (YM_GRAPH=1), mixing zero_grad(set_to_none=True) and in-place zero_grad(set_to_none=False) across the
    eager, capture and replay steps.  The keep-and-add-back of the previous sum runs eagerly around the replayed
    backward, so every step's .grad equals (number of backwards since the last zeroing) x the single-step
    gradient of the same inputs — never a stale sum from the captured step, never a dropped one."""
    from oracle import model as om
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    cfg = om.load_cfg("n")
    _, _, P = om.build(cfg)
    b = {k: v.cuda() for k, v in synth_batch(2, 256, seed=21).items()}
    os.environ["YM_GRAPH"] = "0"
    m0 = build_yolo11(cfg, ch=1, nc=5)
    m0.load_state_dict(P)
    m0 = m0.cuda().train()
    bufs = {k: v.clone() for k, v in m0.state_dict().items()}
    single = _step(m0, v8DetectionLoss(m0), b)[3]
    os.environ["YM_GRAPH"] = "1"
    try:
        m = build_yolo11(cfg, ch=1, nc=5)
        m.load_state_dict(P)
        m = m.cuda().train()
        crit = v8DetectionLoss(m)
        # (zeroing before the step: None = none, True = set_to_none, False = in-place; backwards in the step)
        plan = [(True, 1), (False, 2), (True, 2), (None, 1), (False, 1), (True, 3)]
        count = 0
        for zero, nb in plan:
            if zero is not None:
                m.zero_grad(set_to_none=zero)
                count = 0
            for _ in range(nb):
                m.load_state_dict(bufs)
                loss, _ = crit(m(b["img"].clone()), b)
                loss.backward()
                count += 1
            torch.cuda.synchronize()
            grads = [p.grad for p in m.parameters() if p.grad is not None]
            assert len(grads) == len(single)
            for i, (g, s) in enumerate(zip(grads, single)):
                torch.testing.assert_close(g, s * count, rtol=1e-5, atol=1e-6 * float(s.abs().max()) * count,
                                           msg=f"step {zero, nb} (count {count}) parameter {i}")
    finally:
        os.environ.pop("YM_GRAPH", None)


def test_eval_graph_replay_matches_eager():
    """The eval forward of a model plan replays as a HIP graph (YM_EVAL_GRAPH, on by default): eager on the
    first call, capture on the second, replay after.  Every replay equals the eager forward bit for bit; an
    in-place weight / running-statistics update is seen by the replay (the graph re-reads the fp32 masters and
    the running statistics); a REPLACED parameter or buffer drops the graph (eager run, then a new capture)."""
    import yaml
    from pathlib import Path
    from models import build_yolo11
    root = Path(__file__).resolve().parents[1] / "yolo-scratch_amd"
    cfg = yaml.safe_load((root / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "n"
    torch.manual_seed(5)
    m = build_yolo11(cfg, ch=1, nc=5).cuda().eval()
    g = torch.Generator().manual_seed(6)
    imgs = [torch.rand(1, 1, 320, 320, generator=g).cuda() for _ in range(4)]

    def run(img):
        with torch.no_grad():
            y, _ = m(img)
        torch.cuda.synchronize()
        return y.clone()

    def eager(img):
        os.environ["YM_EVAL_GRAPH"] = "0"
        try:
            return run(img)
        finally:
            os.environ.pop("YM_EVAL_GRAPH", None)

    ref = [eager(i) for i in imgs]
    out = [run(i) for i in imgs]                  # eager, capture, replay, replay
    plan = next(iter(m.__dict__["_ym_plans"].values()))[0]
    assert "fwd" in plan.__dict__.get("_graphs", {}), "the eval forward was not captured"
    for a, b in zip(ref, out):
        assert torch.equal(a, b)
    # in-place updates: same pointers, the replay reads the new values
    with torch.no_grad():
        m.model[2].cv1.conv.weight.mul_(1.5)
        m.model[3].bn.running_mean.add_(0.1)
    r1 = eager(imgs[0])
    assert not torch.equal(r1, ref[0])
    assert torch.equal(run(imgs[0]), r1)
    g0 = plan.__dict__["_graphs"]["fwd"][0]
    # a replaced buffer: the graph is dropped and captured again over the new pointers
    bn = m.model[4].cv2.bn
    bn.running_var = bn.running_var.detach().clone() * 3.0
    r2 = eager(imgs[1])
    assert torch.equal(run(imgs[1]), r2)          # eager (new pointers)
    assert torch.equal(run(imgs[1]), r2)          # capture
    assert torch.equal(run(imgs[1]), r2)          # replay
    assert plan.__dict__["_graphs"]["fwd"][0] is not g0
