"""Timing of SPPF's pool chain at the s@640 bs64 shape (20x20x256, B 64): the fused one-launch
forms (ym_sppf_fwd / _bwd) against three chained per-pool launches (HIP events, --reps each).
usage: python tools/sppf_bench.py [--reps 20 --h 20 --c 256 --b 64]"""
import argparse
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd")]
import torch
from yolomi._lib import call, stream_ptr


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--h", type=int, default=20)
ap.add_argument("--c", type=int, default=256)
ap.add_argument("--b", type=int, default=64)
a = ap.parse_args()
B, H, W, C = a.b, a.h, a.h, a.c
M = B * H * W
st = stream_ptr()
P = torch.randn(4, M, C, device="cuda")
code = torch.zeros(3, M, C, dtype=torch.uint8, device="cuda")
ybuf = torch.zeros(B, H, W, 4 * C, dtype=torch.float16, device="cuda")
gbuf = torch.randn(B, H, W, 4 * C, device="cuda").bfloat16()
G = torch.zeros(2, M, C, device="cuda")
bs, ld = H * W * 4 * C, 4 * C
sl = lambda t, j: t.data_ptr() + 2 * j * C


def fwd3():
    for j in range(3):
        call("ym_maxpool5_f32_fwd", P[j].data_ptr(), P[j + 1].data_ptr(), code[j].data_ptr(), sl(ybuf, j + 1), bs, ld,
             B, H, W, C, st)


def bwd3():
    call("ym_view_to_f32", sl(gbuf, 3), bs, ld, G[0].data_ptr(), M, C, H * W, st)
    cur = G[0]
    for j in (2, 1):
        nxt = G[(3 - j) % 2]
        call("ym_maxpool5_f32_bwd", code[j].data_ptr(), cur.data_ptr(), sl(gbuf, j), bs, ld, nxt.data_ptr(), None, 0,
             0, 0, B, H, W, C, st)
        cur = nxt
    call("ym_maxpool5_f32_bwd", code[0].data_ptr(), cur.data_ptr(), None, 0, 0, None, gbuf.data_ptr(), bs, ld, 1,
         B, H, W, C, st)


def fwd1():
    call("ym_sppf_fwd", P[0].data_ptr(), code.data_ptr(), sl(ybuf, 1), sl(ybuf, 2), sl(ybuf, 3), bs, ld, None,
         B, H, W, C, st)


def bwd1():
    call("ym_sppf_bwd", code.data_ptr(), sl(gbuf, 1), sl(gbuf, 2), sl(gbuf, 3), bs, ld, gbuf.data_ptr(), bs, ld, 1,
         None, B, H, W, C, st)


print(f"SPPF pools {B}x{H}x{W}x{C}: chained fwd {timed(fwd3, a.reps):.1f} us bwd {timed(bwd3, a.reps):.1f} us | "
      f"fused fwd {timed(fwd1, a.reps):.1f} us bwd {timed(bwd1, a.reps):.1f} us")
