"""Reference point only (not the product path): PyTorch's conv2d (MIOpen on ROCm) on the YOLOv11-s@640
bs64 3x3 / 1x1 layer shapes, fp16 channels-last, forward / input-gradient / weight-gradient, timed with
HIP events — what the vendor library reaches on the same shapes as tools/layer_bench.py's kernels.

usage: python tools/miopen_ref.py [--reps 10]
"""
import argparse

import torch

SHAPES = [  # (cin, cout, k, s, out_h) at bs64
    (128, 128, 3, 1, 80), (64, 64, 3, 1, 80), (128, 128, 3, 2, 80), (128, 64, 3, 1, 80),
    (128, 128, 3, 1, 40), (256, 128, 3, 1, 40), (256, 256, 3, 2, 40), (64, 64, 3, 1, 40),
    (128, 128, 3, 1, 20), (256, 512, 3, 2, 20), (512, 128, 3, 1, 20),
    (192, 256, 1, 1, 80), (384, 256, 1, 1, 40), (768, 512, 1, 1, 20), (512, 512, 1, 1, 20),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    print(f"{'cin':>4} {'cout':>4} k s {'out':>4} {'GFLOP':>7} | {'fwd ms':>7} {'frac':>5} | {'dgrad':>7} {'frac':>5} | "
          f"{'wgrad':>7} {'frac':>5}")
    for cin, cout, k, s, oh in SHAPES:
        ih = oh * s
        x = torch.randn(args.batch, cin, ih, ih, device=dev, dtype=torch.float16).to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.float16) * 0.05).to(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w.requires_grad_(True)
        y = torch.nn.functional.conv2d(x, w, stride=s, padding=k // 2)
        dy = torch.randn_like(y)
        fl = 2.0 * args.batch * oh * oh * cout * cin * k * k
        res = []
        for kind in ("fwd", "dgrad", "wgrad"):
            def run():
                if kind == "fwd":
                    torch.nn.functional.conv2d(x, w, stride=s, padding=k // 2)
                elif kind == "dgrad":
                    torch.nn.grad.conv2d_input(x.shape, w, dy, stride=s, padding=k // 2)
                else:
                    torch.nn.grad.conv2d_weight(x, w.shape, dy, stride=s, padding=k // 2)
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            res.append((ms, fl / (ms * 1e-3) / 2.5e15))
        print(f"{cin:4d} {cout:4d} {k} {s} {oh:4d} {fl / 1e9:7.1f} | " +
              " | ".join(f"{ms:7.3f} {fr:5.2f}" for ms, fr in res), flush=True)


if __name__ == "__main__":
    main()
