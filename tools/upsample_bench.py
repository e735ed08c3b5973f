"""Times ym_upsample2_fwd / ym_upsample2_bwd (accumulating) at the s@640 bs64 head shapes (model.11: 512 ch
20x20 -> 40x40 into a 768-channel concat, model.14: 256 ch 40x40 -> 80x80 into 384) with HIP events.
usage: python3 tools/upsample_bench.py [--reps 50]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-scratch_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch
    from yolomi._lib import call
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for n, h, w, c, yc in ((64, 20, 20, 512, 768), (64, 40, 40, 256, 384)):
        x = torch.randn(n, h, w, c, device=dev).half()
        y = torch.empty(n, 2 * h, 2 * w, yc, device=dev).half()
        dx = torch.randn(n, h, w, c, device=dev).bfloat16()
        dy = torch.randn(n, 2 * h, 2 * w, yc, device=dev).bfloat16()
        runs = {"fwd": lambda: call("ym_upsample2_fwd", x.data_ptr(), h * w * c, c, y.data_ptr(), 4 * h * w * yc, yc,
                                    n, h, w, c, None),
                "bwd": lambda: call("ym_upsample2_bwd", dy.data_ptr(), 4 * h * w * yc, yc, dx.data_ptr(), h * w * c, c,
                                    n, h, w, c, 1, None)}
        for k, f in runs.items():
            for _ in range(3):
                f()
            e0.record(s)
            for _ in range(args.reps):
                f()
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            byts = n * h * w * c * 2 * (5 if k == "fwd" else 6)   # fwd: x + 4x y; bwd: 4x dy + dx read + write
            print(f"{k} {c}ch {h}x{w}: {us:7.1f} us  {byts / us / 1e3:6.0f} GB/s")


if __name__ == "__main__":
    main()
