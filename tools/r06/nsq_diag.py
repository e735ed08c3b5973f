"""Diagnostic: per-part head errors (box 64 channels / class channels) and loss items of the GPU and of the rounding
model vs the fp32 oracle, for a non-square odd batch and a square batch of the same images' statistics."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd"), str(ROOT / "tests")):
    sys.path.insert(0, p)


def main():
    import torch
    from test_gpu_model import _seeded_model, _emulated_heads, rel
    from test_gpu_network import _oracle_step
    from oracle import loss as ol
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    for (h, w, bs, seed) in [(96, 160, 3, 19), (160, 96, 3, 19), (128, 128, 3, 19), (96, 160, 3, 23), (96, 160, 2, 19)]:
        b = synth_batch(bs, 128, seed=seed)
        b["img"] = torch.rand(bs, 1, h, w, generator=torch.Generator().manual_seed(seed))
        m = _seeded_model("s").train()
        gb = {k: v.cuda() for k, v in b.items()}
        heads = m(gb["img"])
        loss, items = v8DetectionLoss(m)(heads, gb)
        ref_heads, rl, ri, _, _ = _oracle_step("s", b)
        emu = _emulated_heads("s", b["img"])
        cpu_b = {k: v for k, v in b.items() if k != "img"}
        el, ei = ol.v8_loss([x.detach() for x in emu], cpu_b)
        gl, gi = ol.v8_loss([x.detach().cpu().float() for x in heads], cpu_b)
        out = [f"{h}x{w} bs{bs} seed{seed}:"]
        for i in range(3):
            g, r, e = heads[i].detach().cpu().float(), ref_heads[i], emu[i]
            out.append(f" L{i} box {rel(g[:, :64], r[:, :64]):.4f}/{rel(e[:, :64], r[:, :64]):.4f}"
                       f" cls {rel(g[:, 64:], r[:, 64:]):.4f}/{rel(e[:, 64:], r[:, 64:]):.4f}")
        print("".join(out))
        print(f"   items gpu-fused {[round(float(x), 4) for x in items]}  oracle-loss-on-gpu-heads {[round(float(x), 4) for x in gi]}"
              f"  emu {[round(float(x), 4) for x in ei]}  ref {[round(float(x), 4) for x in ri]}", flush=True)


if __name__ == "__main__":
    main()
