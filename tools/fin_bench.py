"""Per-layer timing of the BatchNorm finalize launches (forward ym_bn_finalize over the conv's stat
rows, backward ym_bn_bwd_finalize over the statistics pass's rows) of a YOLOv11 plan, replayed in
isolation after one training step (HIP events, --reps back-to-back launches each).  Prints the
partial-row counts and the summed time; run under YM_BN_FIN1=0 / default for the A/B.

usage: python tools/fin_bench.py [--scale s --imgsz 640 --batch 64 --reps 20]"""
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
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import yaml
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from yolomi._lib import call, lib, stream_ptr
    from yolomi.graph import ConvBN, _p

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
    ws = plan.bn_ws.data_ptr()
    tot = [0.0, 0.0]
    gs = []
    for op in plan.ops:
        if type(op) is not ConvBN:
            continue
        bn = op.m.bn
        sc, sh, mu, rs = (op.bnv[j].data_ptr() for j in range(4))
        Gb = lib().ym_bn_bwd_blocks(op.M, op.co)
        gs.append((op.G, Gb))
        rm, rv = bn.running_mean.clone(), bn.running_var.clone()
        launches = [
            lambda: call("ym_bn_finalize", op.ps[0].data_ptr(), op.ps[1].data_ptr(), op.G, op.co, float(op.M),
                         _p(bn.weight), _p(bn.bias), rm.data_ptr(), rv.data_ptr(), None, float(bn.momentum),
                         float(bn.eps), sc, sh, mu, rs, ws, st),
            lambda: call("ym_bn_bwd_finalize", op.ps[0].data_ptr(), op.ps[1].data_ptr(), Gb, op.co, float(op.M),
                         _p(bn.weight), rs, None, None, 0, op.coef.data_ptr(), ws, st),
        ]
        for j, fn in enumerate(launches):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for k in range(args.reps + 2):
                if k == 2:
                    e0.record()
                fn()
            e1.record()
            torch.cuda.synchronize()
            tot[j] += e0.elapsed_time(e1) / args.reps * 1e3
    n = len(gs)
    print(f"{n} layers; fwd rows {sorted(set(g for g, _ in gs))}; bwd rows {sorted(set(g for _, g in gs))}")
    print(f"finalize us per step: fwd {tot[0]:.0f} ({tot[0] / n:.1f}/layer)  bwd {tot[1]:.0f} ({tot[1] / n:.1f}/layer)")


if __name__ == "__main__":
    main()
