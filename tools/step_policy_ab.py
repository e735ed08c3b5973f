"""In-step A/B of an experimental library policy (an extern "C" setter of yolomi_experimental.h; run with
YOLOMI_LIB=.../libyolomi_exp.so): the s@640 bs64 training step (forward + fused loss + backward + FusedAdamW) timed
per variant, variants interleaved over rounds in one process (cdna_hip_programming.md §5.4 rule 24).  Measurement
only, never a bench number.

usage: YOLOMI_LIB=$PWD/yolo-scratch_amd/libyolomi_exp.so python tools/step_policy_ab.py SETTER --variants 0 1
"""
import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("setter")
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    import torch
    import yaml
    from yolomi._lib import lib
    from yolomi.optim import FusedAdamW
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    setter = getattr(lib(), args.setter)
    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    torch.manual_seed(0)
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
    crit = v8DetectionLoss(model, tal_topk=10)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=5e-4, max_grad_norm=10.0)
    batches = [prepare_batch(synth_batch(64, 640, seed=i), dev) for i in range(2)]

    def run(n):
        for i in range(n):
            b = batches[i % 2]
            opt.zero_grad(set_to_none=True)
            loss, _ = crit(model(b["img"]), b)
            loss.backward()
            opt.step()

    for v in args.variants:
        setter(v)
        run(3)
    torch.cuda.synchronize()
    res = {v: [] for v in args.variants}
    for _ in range(args.rounds):
        for v in args.variants:
            setter(v)
            run(2)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            run(args.steps)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / args.steps)
    setter(0)
    base = statistics.median(res[args.variants[0]])
    for v, t in res.items():
        m = statistics.median(t)
        print(f"{args.setter} {v}: {m:7.3f} ms/step  {64e3 / m:7.1f} img/s  ({100 * (m - base) / base:+5.2f} %)  "
              f"[{' '.join(f'{x:.3f}' for x in t)}]", flush=True)


if __name__ == "__main__":
    main()
