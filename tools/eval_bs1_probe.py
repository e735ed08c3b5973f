"""Where a bs-1 eval batch's time goes (s@640, the eval forward replayed as a HIP graph): wall time per batch of
(1) model(img) alone, synchronised; (2) model(img) + Detect decode; (3) the end-to-end path of tools/infer_bench.py
(+ decode_predictions_for_metrics, which syncs); and the host time to enqueue (1) without a sync.

usage: python tools/eval_bs1_probe.py [--reps 200]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    import yaml
    from models import build_yolo11
    import train_yolo11_cuda as T
    from yolomi.graph import run_model

    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    torch.manual_seed(0)
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).eval()
    img = torch.rand(args.batch, 1, 640, 640, device=dev)

    def wall(fn, sync_each=True):
        with torch.no_grad():
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                fn()
                if sync_each:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.reps * 1e3

    res = {}
    res["run_model only (plan forward + head clone)"] = wall(lambda: run_model(model, img))
    res["model(img) (+ Detect decode)"] = wall(lambda: model(img))
    res["model(img) + decode_predictions_for_metrics"] = wall(
        lambda: T.decode_predictions_for_metrics(model(img)[0].transpose(1, 2), 640, 0.25, 0.45, dev))
    # host enqueue time of model(img), GPU left running (no sync inside the loop)
    with torch.no_grad():
        torch.cuda.synchronize()
        h = []
        for _ in range(50):
            t0 = time.perf_counter()
            model(img)
            h.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
    res["host enqueue of model(img) (median)"] = sorted(h)[len(h) // 2] * 1e3
    plan = next(iter(model.__dict__["_ym_plans"].values()))[0]
    with torch.no_grad():
        t0 = time.perf_counter()
        for _ in range(200):
            plan._graph_key()
        res["Plan._graph_key() host time"] = (time.perf_counter() - t0) / 200 * 1e3
    for k, v in res.items():
        print(f"{v:8.3f} ms  {k}")


if __name__ == "__main__":
    main()
