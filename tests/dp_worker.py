"""Worker for tests/test_gpu_dp_world2.py: one rank of a 2-process data-parallel run on ONE GPU
(torchrun, YM_DIST_BACKEND=gloo, YM_DIST_DEVICE=0 — RCCL refuses two ranks on one device; the 8-GPU
RCCL run is the driver's).  Not a test module (no test_ prefix): the test launches it.

Per rank, on the real YOLOv11-n plan at 256x256 (models/, losses/, yolomi.dist.GradSync):
* gradients — two input shapes (bs2 and a partial bs1 last batch: two plans, each with its own
  buckets), two backwards each (the first does one plain collective and attaches the plan's hook, the
  second all-reduces its ~8 MB buckets from the backward hook, issued from the side stream after the
  scheduler streams): saves the synced flat gradient of both iterations and the same rank's local
  gradient from an identical model without DP;
* validation — train_yolo11_cuda.validate under DP (each rank its own val batches, detections gathered
  to rank 0, metrics broadcast) after sync_buffers, and on rank 0 the same function with dp=None over
  every rank's batches: the metrics dicts are saved for the test to compare.
usage: python -m torch.distributed.run --nproc-per-node 2 ... tests/dp_worker.py OUTDIR
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def seeded(scale):
    from oracle import model as om
    from models import build_yolo11
    cfg = om.load_cfg(scale)
    _, _, P = om.build(cfg)
    m = build_yolo11(cfg, ch=1, nc=5)
    m.load_state_dict(P)
    return m.cuda().train()


def flat_grad(m):
    return torch.cat([p.grad.detach().reshape(-1).float().cpu() for p in m.parameters() if p.grad is not None])


def main():
    out = Path(sys.argv[1])
    from yolomi import dist as ydist
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    import train_yolo11_cuda as T
    ctx = ydist.init_from_env()
    assert ctx is not None and ctx.world == 2, "launch with torchrun --nproc-per-node 2"
    rank = ctx.rank
    torch.cuda.set_device(0)
    m_dp, m_ref = seeded("n"), seeded("n")
    c_dp, c_ref = v8DetectionLoss(m_dp), v8DetectionLoss(m_ref)
    dp = ydist.GradSync(m_dp, ctx)
    dp.broadcast_state()
    res = {}
    for case, bs in (("full", 2), ("partial", 1)):
        b = {k: v.cuda() for k, v in synth_batch(bs, 256, seed=100 + 10 * rank + bs).items()}
        m_ref.zero_grad(set_to_none=True)
        loss, _ = c_ref(m_ref(b["img"]), b)
        loss.backward()
        torch.save(flat_grad(m_ref), out / f"{case}_local_r{rank}.pt")
        for it in range(2):
            m_dp.zero_grad(set_to_none=True)
            loss, _ = c_dp(m_dp(b["img"]), b)
            loss.backward()
            dp.sync()
            torch.save(flat_grad(m_dp), out / f"{case}_dp{it}_r{rank}.pt")
        plan = m_dp.__dict__["_ym_last_plan"]
        bk = dp.buckets.get(id(plan))
        res[case] = {"buckets": len(bk.ranges) if bk is not None else 0,
                     "hooked": plan.grad_hook is not None, "side_stream": plan.side_stream is not None}
    # validation under DP (rank r: its own 3 batches of 2 images) vs world = 1 over every rank's batches
    dp.sync_buffers()
    vals = [T._SyntheticLoader(3, 2, 256, seed=7000 + 1000 * r) for r in range(2)]
    m_dp.eval()
    vm = T.validate(m_dp, vals[rank], c_dp, torch.device("cuda", 0), dp=dp)
    res["val_dp"] = vm
    if rank == 0:
        class Both:
            def __len__(self):
                return 6

            def __iter__(self):
                for r in range(2):
                    yield from vals[r]
        res["val_world1"] = T.validate(m_dp, Both(), c_dp, torch.device("cuda", 0), dp=None)
    (out / f"res_r{rank}.json").write_text(json.dumps(res))
    import torch.distributed as dist
    dist.barrier()                    # rank 1 waits for rank 0's world-1 validation before tearing down
    ydist.shutdown()


if __name__ == "__main__":
    main()
