"""Times ym_prep_weights (the once-per-step fp32 -> fp16/bf16 weight conversion) over a model plan's
whole weight table: python3 tools/prep_bench.py [--scale s] [--reps 50]."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-scratch_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="s")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch
    import yaml
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from yolomi._lib import stream_ptr

    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = args.scale
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
    crit = v8DetectionLoss(model)
    b = {k: v.to(dev) for k, v in synth_batch(2, 640, seed=1).items()}
    loss, _ = crit(model(b["img"]), b)
    loss.backward()
    torch.cuda.synchronize()
    ws = model.__dict__["_ym_last_plan"].weights
    st = stream_ptr(dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(5):
        ws.refresh(st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.reps):
        ws.refresh(st)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.reps
    n_t = sum(t.numel() for _, _, t, _ in ws.items if t is not None)
    byts = ws.total * 4 + ws.total * 2 + n_t * 2        # fp32 read once (ideal) + fp16 + bf16 writes
    print(f"prep_weights: {len(ws.items)} entries, {ws.total} elements, {us:.1f} us/launch, "
          f"{byts / us / 1e6:.2f} TB/s algorithmic")


if __name__ == "__main__":
    main()
