"""Per-layer timing of the conv kernels (fwd / dgrad / wgrad) of a YOLOv11 plan on the GPU.

Builds the model at the bench configuration, runs one training step to populate every buffer,
then replays each ConvBN's three conv launches in isolation (HIP events on the plan's stream)
and prints achieved TFLOP/s per layer against the 2.5 PFLOP/s dense 16-bit MFMA peak.

usage: python tools/layer_bench.py [--scale s --imgsz 640 --batch 64 --reps 10]
"""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="s")
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", type=int, nargs="*", help="plan op indices to time (default: every ConvBN)")
    ap.add_argument("--hpipe", type=int, default=-1, help="ym_conv_set_hpipe policy for this run (A/B)")
    ap.add_argument("--pipe", type=int, default=-1, help="ym_conv_set_pipe policy for this run (A/B)")
    ap.add_argument("--halo", type=int, default=-1, help="ym_conv_set_halo policy for this run (A/B)")
    ap.add_argument("--direct", type=int, default=-1, help="ym_conv_set_direct policy for this run (A/B)")
    ap.add_argument("--set", nargs="*", default=[], help="other library setters for this run, NAME=VALUE "
                                                        "(e.g. ym_pipe_set_exp=1)")
    ap.add_argument("--names", action="store_true", help="append each launch's kernel instance (ym_conv_kernel)")
    ap.add_argument("--seq-out", help="counter-pass mode: write the (op, kind, k, flops, launches) order of the "
                                      "timed groups here and separate the groups with a marker kernel "
                                      "(tools/pmc_layers.py splits a rocprofv3 --pmc pass on the markers)")
    args = ap.parse_args()
    import torch
    import yaml
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from yolomi._lib import call, stream_ptr
    from yolomi.graph import ConvBN

    from yolomi._lib import lib
    lib().ym_conv_set_hpipe(args.hpipe)
    lib().ym_conv_set_pipe(args.pipe)
    for kv in args.set:
        name, val = kv.split("=")
        getattr(lib(), name)(int(val))
    lib().ym_conv_set_halo(args.halo)
    lib().ym_conv_set_direct(args.direct)
    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = args.scale
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
    crit = v8DetectionLoss(model)
    b = {k: v.to(dev) for k, v in synth_batch(args.batch, args.imgsz, seed=1).items()}
    loss, _ = crit(model(b["img"]), b)
    loss.backward()
    torch.cuda.synchronize()
    plan = model.__dict__["_ym_last_plan"]
    st = stream_ptr(dev)
    ws = plan.wgrad_ws()
    rows = []
    tot = [0.0, 0.0, 0.0]
    seq = []
    marker = torch.zeros(1, device=dev)

    def sep(n=1):
        for _ in range(n):
            marker.add_(1.0)              # one elementwise torch kernel: the group separator of a counter pass
    if args.seq_out:
        torch.cuda.synchronize()
        sep(3)                            # start marker: three separators in a row
    for i, op in enumerate(plan.ops):
        if type(op) is not ConvBN or (args.only and i not in args.only):
            continue
        d = op.desc
        fl = op.flops()
        ms = []
        for kind in ("fwd", "dgrad", "wgrad"):
            if kind == "dgrad" and not plan.needs_grad(op.x):
                ms.append(0.0)
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for r in range(args.reps + 2):
                if r == 2:
                    e0.record()
                if kind == "fwd":
                    call("ym_conv_fwd", ctypes.byref(d), op.x.ptr(), op.wf.data_ptr(), op.z.data_ptr(), None,
                         op.ps[0].data_ptr(), op.ps[1].data_ptr(), st)
                elif kind == "dgrad":
                    call("ym_conv_dgrad", ctypes.byref(d), op.z.data_ptr(), op.wt.data_ptr(), op.x.gptr(), st)
                else:
                    call("ym_conv_wgrad", ctypes.byref(d), op.z.data_ptr(), op.x.ptr(), ws.data_ptr(),
                         ws.numel() * 4, plan.gptr(op.m.conv.weight), 0, st)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1) / args.reps)
            if args.seq_out:
                sep()
                seq.append({"op": i, "kind": kind, "k": d.k, "s": d.stride, "cin": d.cin, "cout": d.cout,
                            "out": [d.oh, d.ow], "flops": fl, "launches": args.reps + 2})
        for j in range(3):
            tot[j] += ms[j]
        tf = [fl / (m * 1e-3) / 1e12 if m > 0 else 0.0 for m in ms]
        # binding-roof fraction per kernel: algorithmic bytes (16-bit tensors read/written once)
        xin = args.batch * d.h * d.w * d.cin * 2
        yout = args.batch * d.oh * d.ow * d.cout * 2
        wb = d.cout * d.cin * d.k * d.k * 2
        byts = [xin + wb + yout, yout + wb + xin, yout + xin + 2 * wb]
        frac = []
        for m, b in zip(ms, byts):
            t_floor = max(fl / 2.5e15, b / 8e12)
            frac.append(t_floor / (m * 1e-3) if m > 0 else 0.0)
        names = []
        if args.names:
            for dr in range(3):
                b_ = ctypes.create_string_buffer(96)
                lib().ym_conv_kernel(ctypes.byref(d), dr, b_, 96)
                names.append(b_.value.decode())
        rows.append((i, d.cin, d.cout, d.k, d.stride, d.oh, d.ow, fl / 1e9, ms, tf, frac,
                     "hbm" if byts[0] / 8e12 > fl / 2.5e15 else "mfma", names))
    print(f"{'op':>4} {'cin':>4} {'cout':>4} k s {'out':>7} {'GFLOP':>7} roof | {'fwd ms':>7} {'TF/s':>5} {'frac':>5} | "
          f"{'dgrad':>7} {'TF/s':>5} {'frac':>5} | {'wgrad':>7} {'TF/s':>5} {'frac':>5}")
    for i, ci, co, k, s, oh, ow, gf, ms, tf, fr, roof, names in rows:
        print(f"{i:4d} {ci:4d} {co:4d} {k} {s} {oh:3d}x{ow:<3d} {gf:7.1f} {roof:>4} | {ms[0]:7.3f} {tf[0]:5.0f} {fr[0]:5.2f} | "
              f"{ms[1]:7.3f} {tf[1]:5.0f} {fr[1]:5.2f} | {ms[2]:7.3f} {tf[2]:5.0f} {fr[2]:5.2f}" +
              ("".join(f" | {n}" for n in names) if names else ""))
    print(f"total ms: fwd {tot[0]:.3f}  dgrad {tot[1]:.3f}  wgrad {tot[2]:.3f}")
    if args.seq_out:
        import json
        Path(args.seq_out).write_text(json.dumps({"batch": args.batch, "imgsz": args.imgsz, "scale": args.scale,
                                                  "groups": seq}))


if __name__ == "__main__":
    main()
