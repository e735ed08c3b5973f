"""Host-side checks of the drop-in model/loss surface (no GPU): graph parse, state_dict keys,
initial buffers/biases, module API, and that the product path refuses CPU tensors."""
import json
import math

import pytest
import torch

from conftest import GOLDEN


@pytest.mark.parametrize("scale", ["n", "s", "m"])
def test_state_dict_matches_reference(scale):
    from models import build_yolo11
    import yaml
    from conftest import PKG
    cfg = yaml.safe_load((PKG / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = scale
    m = build_yolo11(cfg, ch=1, nc=5)
    ref = json.loads((GOLDEN / "structure.json").read_text())[scale]
    assert [[k, list(v.shape), str(v.dtype)] for k, v in m.state_dict().items()] == ref["keys"]
    assert sum(p.numel() for p in m.parameters()) == ref["n_params"]
    assert m.save == ref["save"]
    det = m.model[-1]
    assert det.stride.tolist() == ref["stride"]
    sd = m.state_dict()
    assert float(sd["model.0.bn.running_var"][0]) == pytest.approx(ref["bn_running_var"])
    assert int(sd["model.0.bn.num_batches_tracked"]) == ref["bn_nbt"]
    assert float(sd["model.23.cv3.0.2.bias"][0]) == pytest.approx(ref["detect_bias_cls"])
    assert float(sd["model.23.cv2.0.2.bias"][0]) == pytest.approx(ref["detect_bias_box"])
    assert not det.dfl.conv.weight.requires_grad


def test_seeded_build_matches_reference_init():
    """Same constructor order => same RNG draws: a seeded build reproduces the reference's weights."""
    from models import build_yolo11
    from conftest import PKG
    import yaml
    cfg = yaml.safe_load((PKG / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "n"
    torch.manual_seed(123)
    a = build_yolo11(cfg, ch=1, nc=5).state_dict()
    torch.manual_seed(123)
    b = build_yolo11(cfg, ch=1, nc=5).state_dict()
    assert all(torch.equal(a[k], b[k]) for k in a)
    w = a["model.4.cv2.conv.weight"]
    fan_out = w.shape[0]
    assert abs(float(w.std()) - math.sqrt(2.0 / fan_out)) < 0.02


def test_product_path_refuses_cpu_tensors():
    from models import Conv
    from yolomi import YolomiError
    with pytest.raises(YolomiError):
        Conv(8, 8, 3)(torch.zeros(1, 8, 4, 4))


def test_loss_surface():
    import losses
    for name in ("v8DetectionLoss", "BboxLoss", "TaskAlignedAssigner", "bbox_iou", "bbox2dist", "make_anchors",
                 "dist2bbox"):
        assert hasattr(losses, name)
    b1 = torch.tensor([[0.0, 0.0, 2.0, 2.0]])
    b2 = torch.tensor([[1.0, 1.0, 3.0, 3.0]])
    assert float(losses.bbox_iou(b1, b2, xywh=False)) == pytest.approx(1 / 7, rel=1e-5)


def _model(scale="n"):
    from models import build_yolo11
    import yaml
    from conftest import PKG
    cfg = yaml.safe_load((PKG / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = scale
    return build_yolo11(cfg, ch=1, nc=5)


def _adamw_steps(model, n=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=5e-4)
    for _ in range(n):
        for p in model.parameters():
            if p.requires_grad:
                p.grad = torch.randn(p.shape, generator=g)
        opt.step()
    return opt


def test_checkpoint_roundtrip_and_resume(tmp_path):
    """last.pt as written by the build (the reference's dict, train_yolo11_cuda.py:628-636) resumes
    into a fresh model + AdamW with the reference's procedure (:576-586): weights, optimizer moments
    and epoch/best bookkeeping identical."""
    import train_yolo11_cuda as T
    m = _model()
    opt = _adamw_steps(m)
    ck = T.make_checkpoint(4, m, opt, {"loss": 1.5}, {"loss": 2.0, "mAP50": 0.25}, 2.0, 0.25)
    assert list(ck) == ["epoch", "model_state_dict", "optimizer_state_dict", "train_metrics", "val_metrics",
                        "best_loss", "best_mAP50"]
    torch.save(ck, tmp_path / "last.pt")
    m2 = _model()
    opt2 = torch.optim.AdamW(m2.parameters(), lr=1e-3, weight_decay=5e-4)
    ep, bl, bm = T.resume_checkpoint(tmp_path / "last.pt", m2, opt2, torch.device("cpu"))
    assert (ep, bl, bm) == (5, 2.0, 0.25)
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k
    s1, s2 = opt.state_dict()["state"], opt2.state_dict()["state"]
    assert s1.keys() == s2.keys()
    for i in s1:
        for k in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(s1[i][k], s2[i][k])


def test_reference_layout_checkpoint_resumes(tmp_path):
    """A checkpoint laid out as the reference writes it — state_dict keys/shapes/dtypes from the
    reference's own model (tests/golden/structure.json), parameter order of its AdamW — loads into the
    build (strict) and the optimizer state follows the same parameter indices."""
    import train_yolo11_cuda as T
    ref = json.loads((GOLDEN / "structure.json").read_text())["s"]
    g = torch.Generator().manual_seed(5)
    sd = {}
    for k, shape, dt in ref["keys"]:
        if dt == "torch.int64":
            sd[k] = torch.tensor(7)
        else:
            sd[k] = torch.randn(shape, generator=g)
    m = _model("s")
    opt_ref = _adamw_steps(_model("s"), n=1, seed=9)        # same module tree => same param indices
    # the reference's evaluate_detections returns numpy scalars (np.sum / np.mean, utils/metrics.py:264-274)
    # and they end up in val_metrics and best_mAP50 (train_yolo11_cuda.py:612-653)
    import numpy as np
    vm = {"loss": 3.5, "precision": 0.5, "recall": 0.25, "mAP50": np.float64(0.375), "mAP50-95": np.float64(0.125)}
    ck = {"epoch": 11, "model_state_dict": sd, "optimizer_state_dict": opt_ref.state_dict(),
          "train_metrics": {"loss": 3.0}, "val_metrics": vm, "best_loss": 3.5, "best_mAP50": np.float64(0.375)}
    torch.save(ck, tmp_path / "ref_last.pt")
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=5e-4)
    ep, bl, bm = T.resume_checkpoint(tmp_path / "ref_last.pt", m, opt, torch.device("cpu"))
    assert (ep, bl, bm) == (12, 3.5, 0.375)
    for k, v in sd.items():
        assert torch.equal(m.state_dict()[k], v), k
    assert len(opt.state_dict()["state"]) == len(opt_ref.state_dict()["state"])


def test_fused_adamw_refuses_cpu_parameters():
    """The fused optimizer has no CPU path: CPU parameters raise instead of silently stepping,
    and its state_dict layout is torch.optim.AdamW's (checkpoint interop)."""
    import torch
    from yolomi import YolomiError
    from yolomi.optim import FusedAdamW
    p = torch.nn.Parameter(torch.randn(4))
    p.grad = torch.randn(4)
    opt = FusedAdamW([p], lr=1e-3, weight_decay=5e-4, max_grad_norm=10.0)
    import pytest
    with pytest.raises(YolomiError):
        opt.step()
    ref = torch.optim.AdamW([torch.nn.Parameter(torch.randn(4))], lr=1e-3, weight_decay=5e-4)
    assert set(opt.state_dict()["param_groups"][0]) == set(ref.state_dict()["param_groups"][0])
