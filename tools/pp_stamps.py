"""Diagnostic: per-phase timestamps (s_memtime, shader cycles) of the ping-pong conv kernel on one layer of the
s@640 bs64 plan (workgroup 0, 8 waves, first 32 K steps): where the cycles of a K step go.
usage: python tools/pp_stamps.py OP"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    sys.path.insert(0, p)


def main():
    op_i = int(sys.argv[1]) if len(sys.argv) > 1 else 73
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
    L = lib()
    L.ym_conv_set_hpipe(0)
    op = plan.ops[op_i]
    d = op.desc
    for mode in [int(v) for v in sys.argv[2:]] or [4]:
      print("=== variant", mode, "(4 normal, 5 no DMA, 6 no fragment reads)")
      for m in (1, mode):
        L.ym_conv_set_pipe_pp(m)
        for _ in range(3):
            call("ym_conv_fwd", ctypes.byref(d), op.x.ptr(), op.wf.data_ptr(), op.z.data_ptr(), None,
                 op.ps[0].data_ptr(), op.ps[1].data_ptr(), st)
        torch.cuda.synchronize()
      report(L)


def report(L):
    buf = (ctypes.c_longlong * (8 * 32 * 8))()
    L.ym_pp_stamps(buf)
    t = [[[buf[(w * 32 + g) * 8 + k] for k in range(8)] for g in range(32)] for w in range(8)]
    t0 = min(t[w][0][0] for w in range(8))
    print("wave: per K step g: load0 issue, wait | mfma0 issue, wait || load1 issue, wait | mfma1 issue, wait (cycles)")
    for w in range(8):
        rows = []
        for g in range(31):
            s = t[w][g] + [t[w][g + 1][0]]
            rows.append(" ".join(f"{s[k + 1] - s[k]:4d}" for k in range(8)))
        print(f"w{w}: " + " || ".join(rows[2:6]))
    for w in range(8):
        steps = [t[w][g + 1][0] - t[w][g][0] for g in range(31)]
        print(f"w{w} mean cycles per K step {sum(steps) / len(steps):.0f}  median {sorted(steps)[15]}")


if __name__ == "__main__":
    main()
