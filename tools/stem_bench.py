"""Times ym_conv_first_fwd (the stem: 1 -> 32, 3x3 s2 on the fp32 image, fp16 z + statistics rows) at s@640
bs64 for several workgroup counts.  usage: python3 tools/stem_bench.py [--blocks 1024 768 ...] [--reps 30]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-scratch_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, nargs="*", default=[1024, 768, 512])
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    import torch
    from yolomi._lib import call
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    n, h, w, co = 64, 640, 640, 32
    oh, ow = h // 2, w // 2
    img = torch.rand(n, h, w, device=dev)
    wt = torch.randn(co, 1, 3, 3, device=dev)
    z = torch.empty(n * oh * ow, co, dtype=torch.float16, device=dev)
    st = torch.empty(2, max(args.blocks), co, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for b in args.blocks:
        f = lambda: call("ym_conv_first_fwd", img.data_ptr(), wt.data_ptr(), z.data_ptr(), st[0].data_ptr(),
                         st[1].data_ptr(), n, h, w, oh, ow, co, 2, 1, b, None)
        for _ in range(3):
            f()
        e0.record(s)
        for _ in range(args.reps):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        byts = img.numel() * 4 + z.numel() * 2
        print(f"blocks {b:5d}: {us:7.1f} us  {byts / us / 1e3:6.0f} GB/s")


if __name__ == "__main__":
    main()
