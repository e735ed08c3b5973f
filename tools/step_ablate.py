"""Wall-time share of each kernel family in the s@640 bs64 training step (measurement only, never a bench number).

The step (forward + fused loss + backward; no optimizer, so the weights stay fixed and every variant runs the same
forward) is timed with a family's library calls dropped: the step's shrink is that family's cost on the critical path
once the other streams' overlap is accounted for — what speeding the family up can win at most.  Variants interleave
over rounds in one process (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/step_ablate.py [--steps 20] [--rounds 3]
"""
import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)

FAMILIES = {
    "none": (),
    "wgrad": ("ym_conv_wgrad",),
    "bn_bwd": ("ym_bn_bwd_reduce", "ym_bn_bwd_finalize", "ym_bn_bwd_apply", "ym_bn_bwd_apply_res",
               "ym_bn_bwd_reduce_fold"),
    "bn_fwd_apply": ("ym_bn_apply",),
    "dgrad": ("ym_conv_dgrad",),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", nargs="*", default=list(FAMILIES))
    args = ap.parse_args()
    import torch
    import yaml
    import yolomi.graph as G
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    torch.manual_seed(0)
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
    crit = v8DetectionLoss(model, tal_topk=10)
    batches = [prepare_batch(synth_batch(64, 640, seed=i), dev) for i in range(2)]
    real_call = G.call
    skip = set()

    def call(name, *a):
        if name in skip:
            return
        real_call(name, *a)
    G.call = call

    def run(n):
        for i in range(n):
            b = batches[i % 2]
            model.zero_grad(set_to_none=True)
            loss, _ = crit(model(b["img"]), b)
            loss.backward()

    run(3)
    torch.cuda.synchronize()
    res = {k: [] for k in args.only}
    for _ in range(args.rounds):
        for k in args.only:
            skip.clear()
            skip.update(FAMILIES[k])
            run(2)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            run(args.steps)
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / args.steps)
    base = statistics.median(res["none"]) if "none" in res else None
    for k, v in res.items():
        m = statistics.median(v)
        extra = f"  (step shrinks {base - m:6.3f} ms, {100 * (base - m) / base:5.1f} %)" if base else ""
        print(f"{k:14s} {m:7.3f} ms/step  [{' '.join(f'{x:.3f}' for x in v)}]{extra}", flush=True)


if __name__ == "__main__":
    main()
