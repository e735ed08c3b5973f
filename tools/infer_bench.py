"""Inference benchmark (BASELINE.json configs[4]): YOLOv11-s 640x640 at bs=1 and bs=128.

Two measurements per batch size, inputs resident in HBM:
  * end to end: eval forward (HIP plan, Detect.inference decode) + decode_predictions_for_metrics
    on the anchor-major view of y (one batched decode+NMS launch pair, one host sync) — wall time
    per batch and images/s;
  * postprocess alone: ym_decode_nms on the SURVEY §8(d) NMS workload (anchor-major (B, 8400, 9),
    boxes clustered around 10 objects per image, scores sigmoid(1.5 randn - 2): ~6.7k candidates
    above conf 0.25 per image) timed with HIP events on the launch stream — us per image — and its
    keep-lists checked bit-exact against the CPU oracle (oracle/post.py, the reference's decode /
    nms_simple restated) on every image.
Random-init weights (no checkpoints here): the model's own scores sit near sigmoid(-13.8) (Q4), so
its NMS stage is empty and the postprocess numbers come from the synthetic workload.
CPU baseline: the oracle's fp32 eval forward at bs=1 and its decode+NMS on 8 synthetic images, on
this host's cores.  Prints one JSON line per batch size.

usage: python tools/infer_bench.py [--reps 20 --no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(reps):
        out = fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return out, (time.perf_counter() - t0) / reps * 1e3, e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batches", type=int, nargs="*", default=[1, 128])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import yaml
    from models import build_yolo11
    import train_yolo11_cuda as T
    from datasets.synthetic import synth_eval_preds
    from oracle import post as op
    from yolomi import post as ypost

    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    # A/B of a library policy: YM_LIB_SET="ym_conv_set_eval_cfg=2 ..." (process-wide setters, include/yolomi_experimental.h;
    # the measurement-library ones need YOLOMI_LIB=.../libyolomi_exp.so)
    if os.environ.get("YM_LIB_SET"):
        from yolomi._lib import lib as _yl0
        for kv in os.environ["YM_LIB_SET"].split():
            name, val = kv.split("=")
            getattr(_yl0(), name)(int(val))
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    torch.manual_seed(0)
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).eval()
    def cpu_baseline():
        from oracle import model as om
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        layers, save, P = om.build(om.load_cfg("s"))
        img = torch.rand(1, 1, 640, 640)
        with torch.no_grad():
            om.forward(P, layers, save, img, training=False)
            t0 = time.perf_counter()
            for _ in range(3):
                om.forward(P, layers, save, img, training=False)
            fwd_ms = (time.perf_counter() - t0) / 3 * 1e3
        pred = synth_eval_preds(8, 8400, seed=5).numpy()
        t0 = time.perf_counter()
        op.decode(pred, 640, 0.25, 0.45)
        post_ms = (time.perf_counter() - t0) / 8 * 1e3
        return {"value": round(1e3 / (fwd_ms + post_ms), 3), "unit": "images/sec", "cores": torch.get_num_threads(),
               "kind": "port", "sample": f"oracle fp32 eval forward bs=1 ({fwd_ms:.0f} ms) + oracle decode+NMS "
                                         f"({post_ms:.1f} ms/img over 8 synthetic images)"}
    lines = []
    for B in args.batches:
        img = torch.rand(B, 1, 640, 640, device=dev)
        with torch.no_grad():
            def e2e():
                y, _ = model(img)
                return T.decode_predictions_for_metrics(y.transpose(1, 2), 640, 0.25, 0.45, dev)
            # warm-up: the eval plan runs eagerly once, is captured as a HIP graph on its second call and replays from
            # the third on (yolomi.graph Plan._replay) — the one-time capture stays outside the timed batches
            for _ in range(3):
                e2e()
            _, wall_ms, e2e_gpu_ms = timed(e2e, args.reps, st)
            pred = synth_eval_preds(B, 8400, seed=7 + B)
            pd = pred.to(dev)
            out, post_wall, post_gpu = timed(lambda: ypost.decode_nms(pd, 640, 0.25, 0.45), args.reps, st)
        ref = op.decode(pred.numpy(), 640, 0.25, 0.45)
        exact = all(np.array_equal(o["boxes"].cpu().numpy(), rb) and np.array_equal(o["scores"].cpu().numpy(), rs)
                    and np.array_equal(o["labels"].cpu().numpy(), rl) for o, (rb, rs, rl) in zip(out, ref))
        kept = float(np.mean([len(rs) for _, rs, _ in ref]))
        cand = float((pred[..., 4:].max(-1).values > 0.25).sum(-1).float().mean())
        line = {"metric": "inference images/sec, YOLOv11-s 640x640 (eval forward + decode + NMS)",
                "value": round(B / (wall_ms * 1e-3), 2), "unit": "images/sec", "batch": B,
                "ms_per_batch": round(wall_ms, 3),
                # stream span of one batch between events (includes the host-side gaps of the per-batch sync:
                # at bs1 the wall time is host-enqueue bound and varies with the box's CPU)
                "stream_ms_per_batch": round(e2e_gpu_ms, 3), "higher_is_better": True, "dtype": "fp16 conv / fp32 decode",
                "data": "synthetic images; random-init weights",
                "postprocess": {"us_per_image_gpu": round(post_gpu * 1e3 / B, 2), "ms_per_batch_wall": round(post_wall, 3),
                                "candidates_per_image": round(cand, 1), "kept_per_image": round(kept, 1),
                                "bit_exact_vs_oracle": bool(exact)}}
        lines.append(line)
    # the CPU baseline after the GPU timings (its 16 host threads would otherwise share the host with
    # the launch thread of the host-bound bs1 measurement)
    if not args.no_cpu_baseline:
        lines[0]["cpu_baseline"] = cpu_baseline()
    for line in lines:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
