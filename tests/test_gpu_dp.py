"""The bucketed, backward-overlapped gradient all-reduce (yolomi/dist.py) on RCCL, in one process.

A world of one rank still runs every RCCL collective through the real code path (async bucket
launches from the plan's backward hook, wait, average); the averaged gradients must equal the
plain backward's bit for bit.  World sizes > 1 are covered over gloo in test_dist_cpu.py and run
at 8 GPUs by the driver's scaling bench."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("graph", ["0", "1"])
def test_gradsync_rccl_single_rank_matches_plain_backward(graph, monkeypatch):
    """YM_GRAPH=0: eager backward, bucketed all-reduces launched from the backward hook.
    YM_GRAPH=1: the backward replays as a HIP graph (no hooks), one all-reduce after it."""
    import torch.distributed as dist
    from oracle import model as om
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from yolomi import dist as ydist

    monkeypatch.setenv("YM_GRAPH", graph)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        cfg = om.load_cfg("n")
        layers, save, P = om.build(cfg)
        m = build_yolo11(cfg, ch=1, nc=5)
        m.load_state_dict(P)
        m = m.cuda().train()
        crit = v8DetectionLoss(m)
        sync = ydist.GradSync(m, ydist.DPContext(0, 1, 0), bucket_mb=1.0)
        for step in range(3):                 # step 0 attaches the hook, steps 1-2 use buckets
            b = {k: v.cuda() for k, v in synth_batch(2, 256, seed=40 + step).items()}
            for p in m.parameters():
                p.grad = None
            loss, _ = crit(m(b["img"]), b)
            loss.backward()
            plain = m.__dict__["_ym_last_plan"].grad_flat.clone()
            sync.sync()
            torch.cuda.synchronize()
            got = m.__dict__["_ym_last_plan"].grad_flat
            assert torch.equal(got, plain), step
        plan = m.__dict__["_ym_last_plan"]
        if graph == "0":
            assert len(sync.buckets[id(plan)].ranges) > 1
        else:
            assert sync.buckets[id(plan)] is None and plan.graph_active
    finally:
        dist.destroy_process_group()
