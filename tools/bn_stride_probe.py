"""ym_bn_apply on a 160x160 bs64 map with the output / residual as channel slices of a wider concat
buffer (the C3k2 layout: cv1 writes channels 0..2c of a 3c-wide buffer, the Bottleneck adds its input
slice and writes the last c) against the same work on dense buffers, to separate the strided-view cost
from the kernel.  usage: python3 tools/bn_stride_probe.py [--reps 20]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-scratch_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from yolomi._lib import call, stream_ptr
    dev = torch.device("cuda", 0)
    st = stream_ptr(dev)
    B, H, W = 64, 160, 160
    HW, M = H * W, B * H * W
    cases = [  # (name, C, out ld, out channel offset, residual (ld, offset) or None)
        ("64 dense", 64, 64, 0, None),
        ("64 -> ld 96 @0", 64, 96, 0, None),
        ("64 -> ld 128 @0", 64, 128, 0, None),
        ("32 dense", 32, 32, 0, None),
        ("32 -> ld 96 @64", 32, 96, 64, None),
        ("32 + res dense", 32, 32, 0, (32, 0)),
        ("32 + res ld 96 @32 -> ld 96 @64", 32, 96, 64, (96, 32)),
        ("32 + res ld 96 @32 -> dense", 32, 32, 0, (96, 32)),
        ("32 + res dense -> ld 96 @64", 32, 96, 64, (32, 0)),
    ]
    sc = torch.ones(64, device=dev)
    sh = torch.zeros(64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream(dev)
    print(f"{'case':36s} {'us':>8s} {'GB/s alg':>9s}")
    for name, C, old, ooff, res in cases:
        z = torch.randn(M, C, device=dev).half()
        out = torch.empty(M * old, dtype=torch.float16, device=dev)
        rbuf = torch.randn(M * res[0], device=dev).half() if res else None
        rp = (rbuf.data_ptr() + 2 * res[1]) if res else None
        op = out.data_ptr() + 2 * ooff

        def run():
            call("ym_bn_apply", z.data_ptr(), M, C, HW, sc.data_ptr(), sh.data_ptr(), 1, rp,
                 HW * res[0] if res else 0, res[0] if res else 0, op, HW * old, old, None, st)
        for _ in range(3):
            run()
        e0.record(s)
        for _ in range(args.reps):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        byts = M * C * 2 * (3 if res else 2)
        print(f"{name:36s} {us:8.1f} {byts / us / 1e3:9.0f}")
        del z, out, rbuf


if __name__ == "__main__":
    main()
