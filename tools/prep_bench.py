"""ym_prep_weights alone on a model's conv weights (the table a plan's WeightStore builds): average launch time over
--reps launches, HIP events on the launch stream.  --train adds the transposed data-gradient copies (the training
plan's table); without it the forward copies only (the eval plan's).  YOLOMI_LIB picks the library (A/B).

usage: python tools/prep_bench.py [--scale s --train --reps 200]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="s")
    ap.add_argument("--train", action="store_true")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import yaml
    from models import build_yolo11
    from yolomi._lib import WPrepEntry, call, lib, stream_ptr

    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = args.scale
    torch.manual_seed(0)
    model = build_yolo11(cfg, ch=1, nc=5).to(dev)
    ws = [p for p in model.parameters() if p.dim() == 4]
    keep = []
    arr = (WPrepEntry * len(ws))()
    off = 0
    for e, w in zip(arr, ws):
        co, ci, kh, kw = w.shape
        fwd = torch.empty(co, kh, kw, ci, dtype=torch.float16, device=dev)
        t = torch.empty(ci, kh, kw, co, dtype=torch.bfloat16, device=dev) if args.train else None
        keep += [fwd, t]
        e.src, e.dst_fwd, e.dst_t = w.data_ptr(), fwd.data_ptr(), (t.data_ptr() if t is not None else None)
        e.elem_offset, e.cout, e.cin, e.kh, e.kw, e.cout_t = off, co, ci, kh, kw, co
        off += w.numel()
    table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
    st = torch.cuda.current_stream(dev)
    # a forward-only table takes the forward-only launch where the library has it (as WeightStore.refresh does)
    entry = "ym_prep_weights_fwd" if not args.train and hasattr(lib(), "ym_prep_weights_fwd") else "ym_prep_weights"
    for _ in range(10):
        call(entry, table.data_ptr(), len(ws), off, stream_ptr(dev))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.reps):
        call(entry, table.data_ptr(), len(ws), off, stream_ptr(dev))
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / args.reps * 1e3
    print(json.dumps({"scale": args.scale, "train": args.train, "entry": entry, "entries": len(ws), "elements": off,
                      "us_per_launch": round(us, 2)}))


if __name__ == "__main__":
    main()
