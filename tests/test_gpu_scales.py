"""Every model scale of the reference's yaml (n / s / m / l / x, configs/yolo11n_crater.yaml `scales`) trains and
evaluates through the HIP path: one training step (finite loss, finite gradients on every parameter) and one eval
forward (the one-launch eval blocks, finite decoded output of the reference's shape).  The x scale's 96-channel stem
and 384-channel Attention.pe run as channel pieces (conv.hip ch_pieces); their per-layer numerics are checked in
test_gpu_layers.py (x@128)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale", ["n", "s", "m", "l", "x"])
def test_train_step_and_eval_forward_every_scale(scale):
    import yaml
    from pathlib import Path
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    root = Path(__file__).resolve().parents[1] / "yolo-scratch_amd"
    cfg = yaml.safe_load((root / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = scale
    torch.manual_seed(3)
    m = build_yolo11(cfg, ch=1, nc=5).cuda().train()
    crit = v8DetectionLoss(m, tal_topk=10)
    b = prepare_batch(synth_batch(2, 128, seed=4), torch.device("cuda"))
    loss, _ = crit(m(b["img"]), b)
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all(), scale
    bad = [n for n, p in m.named_parameters() if p.grad is None or not torch.isfinite(p.grad).all()]
    assert not [n for n in bad if "dfl" not in n], bad[:5]
    m.eval()
    with torch.no_grad():
        y, maps = m(b["img"])
    torch.cuda.synchronize()
    assert tuple(y.shape) == (2, 4 + 5, (16 * 16 + 8 * 8 + 4 * 4)) and torch.isfinite(y).all(), (scale, y.shape)


@pytest.mark.parametrize("bs,h,w", [(3, 96, 160), (1, 224, 128)])
def test_train_step_and_eval_forward_odd_shapes(bs, h, w):
    """An odd batch and non-square inputs (multiples of the 32-pixel stride): a training step and an eval forward
    whose decoded rows match the anchor count of the three levels."""
    import yaml
    from pathlib import Path
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    root = Path(__file__).resolve().parents[1] / "yolo-scratch_amd"
    cfg = yaml.safe_load((root / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    torch.manual_seed(5)
    m = build_yolo11(cfg, ch=1, nc=5).cuda().train()
    crit = v8DetectionLoss(m, tal_topk=10)
    b = prepare_batch(synth_batch(bs, 128, seed=6), torch.device("cuda"))
    img = torch.rand(bs, 1, h, w, device="cuda")
    loss, _ = crit(m(img), b)
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all()
    m.eval()
    with torch.no_grad():
        y, _ = m(img)
    torch.cuda.synchronize()
    A = sum((h // s) * (w // s) for s in (8, 16, 32))
    assert tuple(y.shape) == (bs, 9, A) and torch.isfinite(y).all(), y.shape
