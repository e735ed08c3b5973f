"""Same-process A/B of an experimental conv_pipe configuration switch (an extern "C" setter that is NOT in
the header) on the s@640 bs64 plan's layers, variants interleaved over rounds.
usage: python tools/pipe_ab.py SETTER --only 6 10 34 --variants 0 1
       python tools/pipe_ab.py SETTER --setter2 SETTER2 --variants 0:0 0:1 2:1   (value pairs for two setters)
"""
import argparse
import ctypes
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("setter")
    ap.add_argument("--only", type=int, nargs="+", required=True)
    ap.add_argument("--variants", nargs="+", default=["0", "1"])
    ap.add_argument("--setter2", default=None, help="a second setter: variants are then 'v1:v2' pairs")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--also", nargs="*", default=[], help="other setters applied first, NAME=VALUE")
    ap.add_argument("--kinds", nargs="+", default=["fwd", "dgrad"], help="fwd / dgrad / wgrad")
    args = ap.parse_args()
    import torch
    import yaml
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from yolomi._lib import call, lib, stream_ptr
    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
    crit = v8DetectionLoss(model)
    b = {k: v.to(dev) for k, v in synth_batch(64, 640, seed=1).items()}
    loss, _ = crit(model(b["img"]), b)
    loss.backward()
    torch.cuda.synchronize()
    plan = model.__dict__["_ym_last_plan"]
    st = stream_ptr(dev)
    s1 = getattr(lib(), args.setter)
    s2 = getattr(lib(), args.setter2) if args.setter2 else None

    def setter(v):
        parts = str(v).split(":")
        s1(int(parts[0]))
        if s2 is not None:
            s2(int(parts[1]) if len(parts) > 1 else 0)
    for kv in args.also:
        name, val = kv.split("=")
        getattr(lib(), name)(int(val))
    res = {}
    for _ in range(args.rounds):
        for i in args.only:
            op = plan.ops[i]
            d = op.desc
            for v in args.variants:
                setter(v)
                # the variant's own statistics rows: a selection setter can move a layer to a kernel with a
                # larger grid than the plan's buffers were sized for (ym_conv_fwd_stat_rows)
                rows = lib().ym_conv_fwd_stat_rows(ctypes.byref(d))
                stats = torch.empty(2, max(rows, 1), d.cout, dtype=torch.float32, device=dev)
                for kind in args.kinds:
                    if kind == "dgrad" and not plan.needs_grad(op.x):
                        continue
                    if kind == "wgrad":
                        lib().ym_conv_wgrad_workspace_size.restype = ctypes.c_size_t
                        nws = lib().ym_conv_wgrad_workspace_size(ctypes.byref(d))
                        ws = torch.empty(max(1, nws // 4), dtype=torch.float32, device=dev)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    for r in range(args.reps + 2):
                        if r == 2:
                            e0.record()
                        if kind == "fwd":
                            call("ym_conv_fwd", ctypes.byref(d), op.x.ptr(), op.wf.data_ptr(), op.z.data_ptr(), None,
                                 stats[0].data_ptr(), stats[1].data_ptr(), st)
                        elif kind == "dgrad":
                            call("ym_conv_dgrad", ctypes.byref(d), op.z.data_ptr(), op.wt.data_ptr(), op.x.gptr(), st)
                        else:
                            call("ym_conv_wgrad", ctypes.byref(d), op.z.data_ptr(), op.x.ptr(), ws.data_ptr(),
                                 ws.numel() * 4, plan.gptr(op.m.conv.weight), 0, st)
                    e1.record()
                    torch.cuda.synchronize()
                    res.setdefault((i, kind, v), []).append(e0.elapsed_time(e1) / args.reps)
    setter(0)
    for i in args.only:
        d = plan.ops[i].desc
        for kind in args.kinds:
            if (i, kind, args.variants[0]) not in res:
                continue
            line = f"op {i:3d} {d.cin:4d}->{d.cout:<4d} k{d.k} s{d.stride} {d.oh}x{d.ow} {kind:5s}:"
            base = statistics.median(res[(i, kind, args.variants[0])])
            for v in args.variants:
                m = statistics.median(res[(i, kind, v)])
                line += f"  v{v} {m * 1e3:7.1f} us ({(m - base) / base * 100:+5.1f}%)"
            print(line)


if __name__ == "__main__":
    main()
