"""Per-layer timing of the BatchNorm streaming kernels of a YOLOv11 plan on the GPU.

After one training step (every buffer populated), each ConvBN's ym_bn_apply, ym_bn_bwd_reduce and
ym_bn_bwd_apply are replayed in isolation (HIP events, --reps launches each) and their achieved
bandwidth is printed against the algorithmic bytes (16-bit tensors read / written once):
apply z + y (+ residual), bwd_reduce dy + z, bwd_apply dy + z + dz.

usage: python tools/bn_bench.py [--scale s --imgsz 640 --batch 64 --reps 10]
"""
import argparse
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
    args = ap.parse_args()
    import torch
    import yaml
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from yolomi._lib import call, stream_ptr
    from yolomi.graph import ConvBN

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
    tot = [0.0, 0.0, 0.0]
    totb = [0.0, 0.0, 0.0]
    print(f"{'op':>4} {'C':>4} {'map':>7} {'MB':>6} | {'apply us':>8} {'GB/s':>5} | {'reduce':>7} {'GB/s':>5} | "
          f"{'bapply':>7} {'GB/s':>5}")
    for i, op in enumerate(plan.ops):
        if type(op) is not ConvBN:
            continue
        sc, sh, mu, rs = (op.bnv[j].data_ptr() for j in range(4))
        y, r = op.y, op.res
        dy = y.gptr()
        scratch = torch.empty_like(op.z)
        e = op.M * op.co * 2
        byts = [2 * e + (e if r else 0), 2 * e, 3 * e]
        launches = [
            lambda: call("ym_bn_apply", op.z.data_ptr(), op.M, op.co, op.HW, sc, sh, op.act,
                         r.ptr() if r else None, r.bs if r else 0, r.ld if r else 0, y.ptr(), y.bs, y.ld, None, st),
            lambda: call("ym_bn_bwd_reduce", dy, y.bs, y.ld, op.z.data_ptr(), op.M, op.co, op.HW, sc, sh, mu, rs,
                         op.act, op.ps[0].data_ptr(), op.ps[1].data_ptr(), st),
            lambda: call("ym_bn_bwd_apply", dy, y.bs, y.ld, op.z.data_ptr(), op.M, op.co, op.HW, sc, sh, mu, rs,
                         op.act, op.coef.data_ptr(), scratch.data_ptr(), st),
        ]
        us = []
        for fn in launches:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for k in range(args.reps + 2):
                if k == 2:
                    e0.record()
                fn()
            e1.record()
            torch.cuda.synchronize()
            us.append(e0.elapsed_time(e1) / args.reps * 1e3)
        for j in range(3):
            tot[j] += us[j]
            totb[j] += byts[j]
        gbs = [bb / (u * 1e-6) / 1e9 for bb, u in zip(byts, us)]
        print(f"{i:4d} {op.co:4d} {y.H:3d}x{y.W:<3d} {e / 1e6:6.1f} | {us[0]:8.1f} {gbs[0]:5.0f} | {us[1]:7.1f} {gbs[1]:5.0f} | "
              f"{us[2]:7.1f} {gbs[2]:5.0f}")
    print(f"total us: apply {tot[0]:.0f} ({totb[0] / tot[0] / 1e3:.0f} GB/s)  reduce {tot[1]:.0f} "
          f"({totb[1] / tot[1] / 1e3:.0f} GB/s)  bwd_apply {tot[2]:.0f} ({totb[2] / tot[2] / 1e3:.0f} GB/s)")


if __name__ == "__main__":
    main()
