"""Gradient agreement of the fused BatchNorm paths with the unfused ones on the real s@640 bs64 step: the
step-1 parameter gradients (same init, same batch) under two environment settings, and the loss after N
steps.  usage: python3 tools/fold_check.py VAR=a,b [steps] [--worst]   e.g. YM_BWD_FOLD=0,1
SELECT=0,2 instead picks the conv kernels as for batch 0 (own) / 2: different kernels, different fp32
accumulation orders, the same arithmetic — the scale of gradient change plain rounding produces."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-scratch_amd"))


def main():
    import torch
    import yaml
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    from yolomi.optim import FusedAdamW
    var, vals = sys.argv[1].split("=")
    vals = vals.split(",")
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    b = prepare_batch(synth_batch(64, 640, seed=0), dev)
    res = []
    from yolomi._lib import lib
    for v in vals:
        if var == "SELECT":     # a legitimate rounding perturbation: conv kernels chosen as for batch v
            lib().ym_conv_set_select_batch(int(v))
        else:
            os.environ[var] = v
        torch.manual_seed(0)
        m = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
        crit = v8DetectionLoss(m, tal_topk=10)
        opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=5e-4, max_grad_norm=10.0)
        losses = []
        for i in range(steps):
            opt.zero_grad(set_to_none=True)
            loss, _ = crit(m(b["img"]), b)
            loss.backward()
            if i == 0:
                g = [p.grad.detach().clone() for p in m.parameters() if p.grad is not None]
                names = [n for n, p in m.named_parameters() if p.grad is not None]
            opt.step()
            losses.append(float(loss.detach()))
        res.append((v, g, losses))
    (va, ga, la), (vb, gb, lb) = res[0], res[1]
    worst = max(float((x - y).norm() / y.norm().clamp_min(1e-30)) for x, y in zip(ga, gb) if y.norm() > 0)
    tot = float(torch.cat([x.flatten() - y.flatten() for x, y in zip(ga, gb)]).norm() /
                torch.cat([y.flatten() for y in gb]).norm())
    print(f"{var} {va} vs {vb}: step-1 gradient rel diff total {tot:.2e}, worst tensor {worst:.2e}; "
          f"loss after {steps}: {la[-1]:.4f} vs {lb[-1]:.4f}")
    if "--worst" in sys.argv:
        rows = sorted(((float((x - y).norm() / y.norm().clamp_min(1e-30)), n, tuple(y.shape), float(y.norm()))
                       for n, x, y in zip(names, ga, gb)), reverse=True)
        for r in rows[:16]:
            print(f"  {r[0]:.2e}  {r[1]}  {r[2]}  |g| {r[3]:.2e}")


if __name__ == "__main__":
    main()
