"""Pipelined implicit GEMM (conv_pipe.hip) vs the 2-stage implicit GEMM on the GPU: outputs, BN
statistics, and timing, on layer shapes of the s@640 bs64 step.  usage: python tools/pipe_check.py"""
import ctypes
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd")]
import torch
from yolomi._lib import ConvDesc, call, lib

SHAPES = [  # n, h, w, cin, cout, k, s
    (64, 80, 80, 128, 128, 3, 1), (64, 160, 160, 128, 128, 3, 2), (64, 80, 80, 128, 64, 3, 1),
    (64, 40, 40, 256, 128, 3, 1), (64, 80, 80, 256, 256, 3, 2), (64, 40, 40, 128, 128, 3, 1),
    (64, 80, 80, 64, 64, 3, 1), (64, 80, 80, 512, 128, 1, 1), (64, 40, 40, 384, 256, 1, 1),
]


def desc(n, h, w, cin, cout, k, s):
    p = k // 2
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    d = ConvDesc()
    d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, oh, ow, cout, k, s, p
    d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * cin, cin, oh * ow * cout, cout
    d.out_f32, d.accumulate = 2, 0
    return d, oh, ow


def run(d, x, wf, wt, dz, dev, reps=0):
    st = torch.cuda.current_stream().cuda_stream
    rows = lib().ym_conv_fwd_stat_rows(ctypes.byref(d))
    y = torch.empty(d.n, d.oh, d.ow, d.cout, dtype=torch.float16, device=dev)
    ss = torch.zeros(rows, d.cout, device=dev)
    sq = torch.zeros(rows, d.cout, device=dev)
    dx = torch.empty(d.n, d.h, d.w, d.cin, dtype=torch.bfloat16, device=dev)
    f = lambda: call("ym_conv_fwd", ctypes.byref(d), x.data_ptr(), wf.data_ptr(), y.data_ptr(), None, ss.data_ptr(),
                     sq.data_ptr(), st)
    b = lambda: call("ym_conv_dgrad", ctypes.byref(d), dz.data_ptr(), wt.data_ptr(), dx.data_ptr(), st)
    f(); b()
    t = []
    for fn in (f, b):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(reps + 2):
            if r == 2:
                e0.record()
            fn()
        e1.record()
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1) / max(reps, 1))
    return y, ss.sum(0), sq.sum(0), dx, t


def main():
    dev = torch.device("cuda")
    ok = True
    only = [int(v) for v in sys.argv[1:]]
    for si, sh in enumerate(SHAPES):
        if only and si not in only:
            continue
        n, h, w, cin, cout, k, s = sh
        d, oh, ow = desc(*sh)
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.randn(n, h, w, cin, device=dev, generator=g).half()
        wf = (torch.randn(cout, k, k, cin, device=dev, generator=g) * (2.0 / (cin * k * k)) ** 0.5).half()
        wt = wf.permute(3, 1, 2, 0).contiguous().bfloat16()
        dz = torch.randn(n, oh, ow, cout, device=dev, generator=g).bfloat16()
        algo_f, algo_b = lib().ym_conv_algo(ctypes.byref(d), 0), lib().ym_conv_algo(ctypes.byref(d), 1)
        lib().ym_conv_set_pipe(0)
        r0 = run(d, x, wf, wt, dz, dev, reps=10)
        lib().ym_conv_set_pipe(2)
        a2f, a2b = lib().ym_conv_algo(ctypes.byref(d), 0), lib().ym_conv_algo(ctypes.byref(d), 1)
        r1 = run(d, x, wf, wt, dz, dev, reps=10)
        lib().ym_conv_set_pipe(-1)
        rel = lambda a, b: float((a.float() - b.float()).abs().max() / b.float().abs().max())
        errs = [rel(r1[0], r0[0]), rel(r1[1], r0[1]), rel(r1[2], r0[2]), rel(r1[3], r0[3])]
        fl = 2 * n * oh * ow * cout * cin * k * k
        good = errs[0] < 2e-3 and errs[1] < 1e-3 and errs[2] < 1e-3 and errs[3] < 1e-2 and torch.isfinite(r1[3].float()).all()
        ok &= bool(good)
        print(f"{sh} algo {algo_f}/{algo_b}->{a2f}/{a2b} err y {errs[0]:.1e} sum {errs[1]:.1e} sq {errs[2]:.1e} dx {errs[3]:.1e} "
              f"| fwd {r0[4][0]:.3f} -> {r1[4][0]:.3f} ms ({fl / r1[4][0] / 1e9 / 2500:.2f} of peak) "
              f"| dgrad {r0[4][1]:.3f} -> {r1[4][1]:.3f} ms ({fl / r1[4][1] / 1e9 / 2500:.2f}) {'OK' if good else 'MISMATCH'}",
              flush=True)
    print("ALL OK" if ok else "MISMATCHES")


if __name__ == "__main__":
    main()
