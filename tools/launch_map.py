"""Per-launch -> layer map of a training step, and the conv / BatchNorm families recomputed from a rocprofv3
kernel trace of exactly those launches.

    # GPU box: record the last step's library calls (one stream, no side stream, as bench.py's probe pass)
    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/launch_map.py record OUT/calls.json
    # anywhere: join the trace with the call list
    python3 tools/launch_map.py join OUT/.../run_kernel_trace.csv OUT/calls.json > layer_map.txt

`record` builds bench.py's workload (YOLOv11-s 640x640 bs64, seed 0, FusedAdamW), warms up on the default 3 +
side streams, then runs the mapped steps with YM_STREAMS=1 YM_SIDE_STREAM=0 (each kernel's duration is its
own) and writes every libyolomi call of the LAST step in issue order with its plan op (index, type, phase,
conv direction, FLOPs).  The step is bracketed in the trace by three marker kernels on each side.
`join` walks the trace's kernels between the markers in dispatch order and assigns each recorded conv / BN
call the kernels it launches (by name, in order); everything else is counted as "other".  The 3x3 family
(fwd / dgrad / wgrad + split-K reduce launches of k=3 Conv blocks) and its fraction of the 2.5 PF MFMA peak
follow from the printed rows, as bench.py's `roofline` does from HIP events.
"""
import collections
import csv
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

PEAK_TF = 2500.0
CONV = r"conv_(direct|direct_quad|hpipe|pipe|halo|gemm)_kernel"
EXPECT = {
    "ym_conv_fwd": [CONV],
    "ym_conv_fwd_bn": [CONV],
    "ym_conv_dgrad": [CONV],
    "ym_conv_wgrad": [r"wgrad(3|1|_generic)_kernel", r"wgrad_reduce_kernel"],
    "ym_bn_finalize": [r"bn_finalize_fused_kernel"],
    "ym_bn_apply": [r"bn_apply_kernel"],
    "ym_bn_bwd_reduce": [r"bn_bwd_reduce_kernel"],
    "ym_bn_bwd_finalize": [r"bn_finalize_fused_kernel"],
    "ym_bn_bwd_apply": [r"bn_bwd_apply_kernel"],
    "ym_bn_bwd_apply_res": [r"bn_bwd_apply_kernel"],
}
MARK = "vectorized_elementwise_kernel"      # the marker: torch's elementwise add on a one-element tensor


def record(out, steps=2, warmup=3):
    import os
    import torch
    import yaml
    import yolomi._lib as L
    import yolomi.graph as G
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    from yolomi.optim import FusedAdamW
    dev = torch.device("cuda", 0)
    cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = "s"
    torch.manual_seed(0)
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
    crit = v8DetectionLoss(model, tal_topk=10)
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=5e-4, max_grad_norm=10.0)
    b = prepare_batch(synth_batch(64, 640, seed=0), dev)

    def step():
        opt.zero_grad(set_to_none=True)
        loss, _ = crit(model(b["img"]), b)
        loss.backward()
        opt.step()
    for _ in range(warmup):
        step()
    # one stream, and the forward BatchNorm finalize as its own launch (as bench.py's family pass times it)
    os.environ.update(YM_STREAMS="1", YM_SIDE_STREAM="0", YM_FOLD="0")
    for _ in range(steps - 1):
        step()
    plan = model.__dict__["_ym_last_plan"]
    calls, cur = [], [None]

    def on_op(i, op, phase):
        d = {"op": i if phase == "fwd" else len(plan.ops) - 1 - i, "type": type(op).__name__, "phase": phase}
        if type(op).__name__ == "ConvBN":
            d.update(k=op.k, s=op.s, ci=op.ci, co=op.co, out=[op.y.H, op.y.W], flops=op.flops())
        cur[0] = d
    orig = L.call
    mods = [m for m in list(sys.modules.values()) if getattr(m, "call", None) is orig]

    def rec(name, *a):
        calls.append({"call": name, **(cur[0] or {"op": None})})
        return orig(name, *a)
    for m in mods:
        m.call = rec
    plan.on_op = on_op
    marker = torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    for _ in range(3):
        marker.add_(1.0)
    step()
    for _ in range(3):
        marker.add_(1.0)
    torch.cuda.synchronize()
    plan.on_op = None
    for m in mods:
        m.call = orig
    Path(out).write_text(json.dumps({"calls": calls, "batch": 64, "imgsz": 640, "scale": "s"}))
    print(f"recorded {len(calls)} calls of one step", file=sys.stderr)


def join(trace, calls_json):
    rows = list(csv.DictReader(open(trace)))
    key = "Dispatch_Id" if "Dispatch_Id" in rows[0] else "Start_Timestamp"
    ks = sorted(rows, key=lambda r: int(r[key]))
    names = [r["Kernel_Name"] for r in ks]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]     # us
    # the step: between the last run of three markers before it and the first run after it
    runs = [i for i in range(len(names) - 2) if all(MARK in names[i + j] for j in range(3))]
    if len(runs) < 2:
        raise SystemExit("markers not found in the trace")
    lo, hi = runs[-2] + 3, runs[-1]
    while MARK in names[lo] and lo < hi:
        lo += 1
    calls = json.loads(Path(calls_json).read_text())["calls"]
    pos, mapped, taken = lo, [], set()
    for c in calls:
        pats = EXPECT.get(c["call"])
        if not pats:
            continue
        us, kn = 0.0, []
        for pat in pats:
            j = pos
            while j < hi and not re.search(pat, names[j]):
                j += 1
            if j >= hi:
                raise SystemExit(f"no kernel for {c['call']} op {c.get('op')} ({pat}) after dispatch {pos}")
            us += dur[j]
            kn.append(re.sub(r"\(.*", "", names[j].replace("ym::(anonymous namespace)::", "").replace("void ", "")))
            taken.add(j)
            pos = j + 1
        mapped.append((c, us, kn))
    other = sum(dur[j] for j in range(lo, hi) if j not in taken)
    fam = collections.defaultdict(lambda: [0.0, 0.0, 0])      # name -> us, flops, launches
    print(f"{'op':>4} {'dir':>5} {'k':>1} {'s':>1} {'cin':>4} {'cout':>4} {'out':>7} {'GFLOP':>7} {'us':>8} "
          f"{'TF/s':>6} {'frac':>5}  kernel")
    for c, us, kn in mapped:
        call = c["call"]
        if call.startswith("ym_conv") and c.get("type") == "ConvBN":
            dr = {"ym_conv_fwd": "fwd", "ym_conv_fwd_bn": "fwd", "ym_conv_dgrad": "dgrad", "ym_conv_wgrad": "wgrad"}[call]
            fl = c["flops"]
            tf = fl / (us * 1e-6) / 1e12
            print(f"{c['op']:4d} {dr:>5} {c['k']} {c['s']} {c['ci']:4d} {c['co']:4d} {c['out'][0]:3d}x{c['out'][1]:<3d} "
                  f"{fl / 1e9:7.1f} {us:8.1f} {tf:6.0f} {tf / PEAK_TF:5.3f}  {' + '.join(kn)}")
            for f in (dr, f"{dr}{c['k']}"):
                fam[f][0] += us
                fam[f][1] += fl
                fam[f][2] += 1
        elif call.startswith("ym_bn"):
            fam["bn"][0] += us
            fam["bn"][2] += 1
        else:
            fam["conv (non-ConvBN)"][0] += us
            fam["conv (non-ConvBN)"][2] += 1
    tot = sum(dur[lo:hi])
    print(f"\nstep kernels {hi - lo}, summed durations {tot / 1e3:.3f} ms (one stream); unattributed {other / 1e3:.3f} ms")
    for f in ("fwd", "dgrad", "wgrad", "fwd3", "dgrad3", "wgrad3", "fwd1", "dgrad1", "wgrad1", "bn", "conv (non-ConvBN)"):
        us, fl, n = fam[f]
        extra = f"  {fl / 1e9:8.1f} GFLOP  {fl / (us * 1e-6) / 1e12:6.1f} TF/s = {fl / (us * 1e-6) / 1e12 / PEAK_TF:.4f} of MFMA" \
            if fl else ""
        print(f"{f:>18}: {us / 1e3:7.3f} ms  {n:4d} launches{extra}")
    c3 = [fam[f] for f in ("fwd3", "dgrad3", "wgrad3")]
    us, fl = sum(x[0] for x in c3), sum(x[1] for x in c3)
    print(f"\n3x3 family (bench.py `roofline`): {fl / 1e9:.0f} GFLOP in {us / 1e3:.3f} ms = "
          f"{fl / (us * 1e-6) / 1e12:.1f} TF/s = {fl / (us * 1e-6) / 1e12 / PEAK_TF:.4f} of the 2.5 PF MFMA peak")


if __name__ == "__main__":
    if sys.argv[1] == "record":
        record(sys.argv[2])
    elif sys.argv[1] == "join":
        join(sys.argv[2], sys.argv[3])
    else:
        raise SystemExit(__doc__)
