"""Host time per phase of the bench's s@640 bs64 step in STEADY STATE (no synchronisation inside the loop): a phase
whose host time is far above its enqueue cost (tools/step_phases.py, which starts each step on an idle GPU) is where
the host blocks on the GPU — the point where a host that should run ahead of the GPU is held back to its pace.

usage: python tools/host_phases.py [--steps 30]
"""
import argparse
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    import yaml
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    from yolomi.optim import FusedAdamW

    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    torch.manual_seed(0)
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
    crit = v8DetectionLoss(model, tal_topk=10)
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=5e-4, max_grad_norm=10.0)
    batches = [prepare_batch(synth_batch(64, 640, seed=i), dev) for i in range(4)]
    names = ["zero_grad", "forward", "loss", "backward", "optimizer"]
    rec = []
    for i in range(8 + args.steps):
        b = batches[i % 4]
        t = [time.perf_counter()]
        opt.zero_grad(set_to_none=True)
        t.append(time.perf_counter())
        preds = model(b["img"])
        t.append(time.perf_counter())
        loss, _ = crit(preds, b)
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        if i >= 8:
            rec.append([(t[k + 1] - t[k]) * 1e3 for k in range(5)])
    torch.cuda.synchronize()
    med = statistics.median
    print(f"steady-state host ms per phase (median of {args.steps} steps, no sync inside the loop):")
    print("  " + "  ".join(f"{n} {med([r[k] for r in rec]):.3f}" for k, n in enumerate(names)))
    print(f"  step {med([sum(r) for r in rec]):.3f}")
    print("  max per phase: " + "  ".join(f"{n} {max(r[k] for r in rec):.3f}" for k, n in enumerate(names)))


if __name__ == "__main__":
    main()
