"""Where the training step's GPU idles at the forward -> loss -> backward transition: host vs GPU time per phase.

Runs the bench's s@640 bs64 step (same model / loss / optimizer / batches as bench.py) and, per step, records a HIP
event AND the host clock at each phase boundary (step start, after model(img), after the loss, after backward(),
after the optimizer).  For each phase it prints the median host time spent enqueueing it and the median GPU time
between its boundary events; the host's lead over the GPU at each boundary (GPU event time - host enqueue time,
both relative to the step's start, GPU clock read by elapsed_time) shows where the GPU can run dry: a lead near zero
means the GPU waited for the host there.

usage: python tools/step_phases.py [--steps 20]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
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
    batches = [prepare_batch(synth_batch(args.batch, 640, seed=i), dev) for i in range(4)]
    st = torch.cuda.current_stream(dev)
    names = ["start", "forward", "loss", "backward", "optimizer"]

    def step(i, rec):
        b = batches[i % 4]
        marks = []

        def mark():
            e = torch.cuda.Event(enable_timing=True)
            e.record(st)
            marks.append((time.perf_counter(), e))
        opt.zero_grad(set_to_none=True)
        mark()
        preds = model(b["img"])
        mark()
        loss, _ = crit(preds, b)
        mark()
        loss.backward()
        mark()
        opt.step()
        mark()
        if rec is not None:
            rec.append(marks)

    for i in range(5):
        step(i, None)
    torch.cuda.synchronize()
    recs = []
    for i in range(args.steps):
        step(5 + i, recs)
        torch.cuda.synchronize()          # one step at a time: the host starts each step with the GPU idle
    host = {n: [] for n in names[1:]}
    gpu = {n: [] for n in names[1:]}
    lead = {n: [] for n in names}
    for marks in recs:
        h0, e0 = marks[0]
        for k in range(1, len(names)):
            host[names[k]].append((marks[k][0] - marks[k - 1][0]) * 1e3)
            gpu[names[k]].append(marks[k - 1][1].elapsed_time(marks[k][1]))
        for k in range(len(names)):
            lead[names[k]].append(e0.elapsed_time(marks[k][1]) - (marks[k][0] - h0) * 1e3)
    med = statistics.median
    print(f"{'phase':10s} {'host ms':>8s} {'gpu ms':>8s}   (median of {args.steps} steps, each started on an idle GPU)")
    for n in names[1:]:
        print(f"{n:10s} {med(host[n]):8.3f} {med(gpu[n]):8.3f}")
    print("GPU behind the host at each boundary (ms, GPU event time - host enqueue time from the step's start):")
    print("  " + "  ".join(f"{n} {med(lead[n]):.3f}" for n in names))


if __name__ == "__main__":
    main()
