"""The fused loss (ym_loss_fwd / ym_loss_bwd) at class counts other than the crater config's 5: 1, 16 (the largest
count loss_partial stages through LDS), 17 (the first it reads from the rows directly) and 80 (COCO), against the
CPU oracle's v8_loss (oracle/loss.py, following yolo_v8_loss.py:372-499) on the same fp32 head maps — assignment
decisions exact, loss / items within 1e-4, head-map gradients within 1e-3 (the golden assigner test's bounds)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nc", [1, 16, 17, 80])
def test_fused_loss_class_counts_vs_oracle(nc):
    import torch.nn as nn
    from models import Detect
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from oracle import loss as ol

    class Stub(nn.Module):
        def __init__(self):
            super().__init__()
            self.det = Detect(nc, (64, 128, 256))
            self.det.stride = torch.tensor([8.0, 16.0, 32.0])

    B, imgsz = 3, 256
    b = synth_batch(B, imgsz, seed=100 + nc, nc=nc)
    batch = {k: b[k] for k in ("batch_idx", "cls", "bboxes")}
    g = torch.Generator().manual_seed(nc)
    feats = [torch.randn(B, 64 + nc, imgsz // s, imgsz // s, generator=g) * 2.0 for s in (8, 16, 32)]

    crit = v8DetectionLoss(Stub().cuda())
    fd = [f.cuda().requires_grad_(True) for f in feats]
    loss, items = crit(fd, {k: v.cuda() for k, v in batch.items()})
    tgi, fg, nm = crit.assignment()
    loss.backward()

    fr = [f.clone().requires_grad_(True) for f in feats]
    rl, ri, inter = ol.v8_loss(fr, batch, nc=nc, return_internals=True)
    rl.backward()

    assert int(inter["fg"].sum()) > 0
    np.testing.assert_array_equal(fg.cpu().numpy().astype(bool), inter["fg"].numpy())
    fgm = inter["fg"]
    np.testing.assert_array_equal(tgi.cpu()[fgm].numpy(), inter["tgi"][fgm].numpy())
    torch.testing.assert_close(items.cpu(), ri, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(loss.detach().cpu(), rl.detach(), rtol=1e-4, atol=1e-6)
    for a, r in zip(fd, fr):
        torch.testing.assert_close(a.grad.cpu(), r.grad, rtol=1e-3, atol=1e-6)


def test_model_80_classes_train_step_and_eval():
    """An 80-class model through the HIP path (ym_head_grad's class rows padded to 8-channel groups): the fused loss
    on the network's own heads equals the oracle's v8_loss on the same heads (1e-4), every gradient is finite, and the
    eval forward decodes (B, 4 + 80, A) finite rows (gradients vs the oracle at nc = 80: test_gpu_network.py
    test_model_80_classes_train_step_vs_oracle).  An image whose plane count differs from the model's ch is refused
    with the reference's Conv2d message."""
    ch = 1
    import yaml
    from pathlib import Path
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    from oracle import loss as ol
    root = Path(__file__).resolve().parents[1] / "yolo-scratch_amd"
    cfg = yaml.safe_load((root / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    torch.manual_seed(8)
    nc = 80
    m = build_yolo11(cfg, ch=ch, nc=nc).cuda().train()
    crit = v8DetectionLoss(m, tal_topk=10)
    b = prepare_batch(synth_batch(2, 160, seed=9, nc=nc, ch=ch), torch.device("cuda"))
    heads = m(b["img"])
    loss, items = crit(heads, b)
    loss.backward()
    torch.cuda.synchronize()
    cpu_b = {k: b[k].cpu() for k in ("batch_idx", "cls", "bboxes")}
    rl, ri = ol.v8_loss([h.detach().float().cpu() for h in heads], cpu_b, nc=nc)
    torch.testing.assert_close(items.cpu(), ri, rtol=1e-4, atol=1e-6)
    bad = [n for n, p in m.named_parameters() if p.grad is None or not torch.isfinite(p.grad).all()]
    assert not [n for n in bad if "dfl" not in n], bad[:5]
    m.eval()
    with torch.no_grad():
        y, _ = m(b["img"])
    torch.cuda.synchronize()
    assert tuple(y.shape) == (2, 4 + nc, 20 * 20 + 10 * 10 + 5 * 5) and torch.isfinite(y).all(), y.shape
    from yolomi.post import decode_nms
    dets = decode_nms(y.transpose(1, 2), 160, 0.001, 0.7)      # 80 class columns through the batched decode + NMS
    assert len(dets) == 2
    from yolomi._lib import YolomiError
    with pytest.raises(YolomiError, match="to have 1 channels, but got 3 channels"):
        m(torch.rand(1, 3, 64, 64, device="cuda"))
