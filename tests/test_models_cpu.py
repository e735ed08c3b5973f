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
