"""Times ym_conv_fwd / ym_conv_dgrad of dense 1x1 layers (synthetic tensors, no model) under several
ym_conv_set_pipe1x1 settings, same process: python3 tools/s1_probe.py --modes 0 1 [--shapes n,h,w,cin,cout ...]."""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-scratch_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--shapes", nargs="+", default=["64,40,40,128,64", "64,80,80,128,128", "64,20,20,256,128",
                                                     "64,80,80,192,256", "64,80,80,512,128"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    from yolomi._lib import ConvDesc, call, lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    L = lib()
    for sh in args.shapes:
        n, h, w, cin, cout = map(int, sh.split(","))
        d = ConvDesc()
        d.n, d.h, d.w, d.cin, d.oh, d.ow, d.cout, d.k, d.stride, d.pad = n, h, w, cin, h, w, cout, 1, 1, 0
        d.x_bs, d.x_ld, d.y_bs, d.y_ld = h * w * cin, cin, h * w * cout, cout
        d.out_f32, d.accumulate = 2, 0
        x = torch.randn(n, h, w, cin, device=dev).half()
        wf = torch.randn(cout, cin, device=dev).half()
        wt = torch.randn(cin, cout, device=dev).bfloat16()
        y = torch.empty(n, h, w, cout, device=dev, dtype=torch.float16)
        dz = torch.randn(n, h, w, cout, device=dev).bfloat16()
        dx = torch.empty(n, h, w, cin, device=dev, dtype=torch.bfloat16)
        res = {}
        for kind in ("fwd", "dgrad"):
            for r in range(args.rounds):
                for m in args.modes:
                    prev = L.ym_conv_set_pipe1x1(m)
                    try:
                        rows = L.ym_conv_fwd_stat_rows(ctypes.byref(d))
                        ss = torch.empty(max(rows, 1), cout, device=dev)
                        sq = torch.empty_like(ss)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        for i in range(args.reps + 2):
                            if i == 2:
                                e0.record()
                            if kind == "fwd":
                                call("ym_conv_fwd", ctypes.byref(d), x.data_ptr(), wf.data_ptr(), y.data_ptr(), None,
                                     ss.data_ptr(), sq.data_ptr(), st)
                            else:
                                call("ym_conv_dgrad", ctypes.byref(d), dz.data_ptr(), wt.data_ptr(), dx.data_ptr(), st)
                        e1.record()
                        torch.cuda.synchronize()
                        t = e0.elapsed_time(e1) * 1e3 / args.reps
                        res[(kind, m)] = min(res.get((kind, m), 1e9), t)
                    finally:
                        L.ym_conv_set_pipe1x1(prev)
            mb = n * h * w * (cin + cout) * 2 / 1e6
            print(f"{sh:>18} {kind:5} {mb:6.0f} MB | " +
                  "  ".join(f"m{m}: {res[(kind, m)]:7.1f} us {mb / res[(kind, m)]:5.2f} TB/s" for m in args.modes),
                  flush=True)


if __name__ == "__main__":
    main()
