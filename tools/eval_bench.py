"""Detection-metrics throughput: utils.metrics.evaluate_packed (HIP) vs the numpy oracle.

Validation-scale synthetic workload: --images images, each with U(0, --max-gt) GT boxes and
~1.5x as many predictions (jittered copies of the GT plus spurious boxes, scores with ties).
GPU: the whole ym_eval_detections chain timed with HIP events on the launch stream (inputs
resident in HBM; host packing excluded).  CPU: oracle/metrics.py on the first --cpu-images
images, scaled to images/s.  Prints one JSON line.

usage: python tools/eval_bench.py [--images 5000 --max-gt 100 --reps 20 --cpu-images 200]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def workload(n_img, max_gt, seed=0):
    rng = np.random.default_rng(seed)
    gc = rng.integers(0, max_gt + 1, n_img)
    ng = int(gc.sum())
    c = rng.random((ng, 2))
    wh = 0.01 + 0.1 * rng.random((ng, 2))
    gb = np.clip(np.concatenate([c - wh / 2, c + wh / 2], 1), 0, 1).astype(np.float32)
    # predictions: every GT once (jittered) + 50 % spurious, per image
    pc = gc + gc // 2
    pb_list, off = [], 0
    for b in range(n_img):
        g = gb[off:off + gc[b]]
        off += gc[b]
        j = g + rng.normal(0, 0.01, g.shape)
        s = rng.random((gc[b] // 2, 4))
        pb_list.append(np.concatenate([j, s]))
    pb = np.concatenate(pb_list).astype(np.float32)
    pb = np.stack([np.minimum(pb[:, 0], pb[:, 2]), np.minimum(pb[:, 1], pb[:, 3]),
                   np.maximum(pb[:, 0], pb[:, 2]), np.maximum(pb[:, 1], pb[:, 3])], 1).astype(np.float32)
    ps = (np.floor(rng.random(len(pb)) * 1000) / 1000).astype(np.float32)
    return pb, ps, pc, gb, gc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=5000)
    ap.add_argument("--max-gt", type=int, default=100)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cpu-images", type=int, default=200)
    args = ap.parse_args()
    from utils import metrics as um
    pb, ps, pc, gb, gc = workload(args.images, args.max_gt)
    dev = torch.device("cuda", 0)
    tpb, tps, tgb = (torch.from_numpy(x).to(dev) for x in (pb, ps, gb))
    r = um.evaluate_packed(tpb, tps, pc.tolist(), tgb, gc.tolist(), 0.25, 0.5)        # warm-up
    torch.cuda.synchronize()
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(args.reps):
        r = um.evaluate_packed(tpb, tps, pc.tolist(), tgb, gc.tolist(), 0.25, 0.5)
    e1.record(st)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.reps
    gpu_ms = e0.elapsed_time(e1) / args.reps
    # CPU oracle on a bounded sample
    from oracle import metrics as omet
    k = args.cpu_images
    npk, ngk = int(pc[:k].sum()), int(gc[:k].sum())
    preds, tgts, po, go = [], [], 0, 0
    for b in range(k):
        preds.append({"boxes": torch.from_numpy(pb[po:po + pc[b]]), "scores": torch.from_numpy(ps[po:po + pc[b]])})
        tgts.append({"boxes": torch.from_numpy(gb[go:go + gc[b]])})
        po += pc[b]
        go += gc[b]
    t0 = time.perf_counter()
    ref = omet.evaluate_detections(preds, tgts, 0.25, 0.5, per_threshold=True)
    cpu_s = time.perf_counter() - t0
    sub = um.evaluate_packed(tpb[:npk], tps[:npk], pc[:k].tolist(), tgb[:ngk], gc[:k].tolist(), 0.25, 0.5)
    parity = (sub["tp50"] == ref["tp50"] and sub["fp50"] == ref["fp50"]
              and np.allclose(sub["ap"], ref["ap"], rtol=1e-12, atol=1e-15))
    print(json.dumps({
        "metric": "evaluate_detections_images_per_s", "value": args.images / (gpu_ms * 1e-3), "unit": "images/s",
        "ms_per_eval": gpu_ms, "wall_ms_per_call": wall * 1e3, "images": args.images,
        "predictions": int(pc.sum()), "gt": int(gc.sum()), "mAP50": r["mAP50"], "mAP50-95": r["mAP50-95"],
        "cpu_baseline": {"value": k / cpu_s, "unit": "images/s", "cores": 1, "kind": "port",
                         "sample": f"oracle/metrics.py on the first {k} images"},
        "parity_on_sample": bool(parity)}))


if __name__ == "__main__":
    main()
