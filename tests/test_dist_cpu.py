"""Data-parallel layer (yolomi/dist.py) at world size 2 over gloo on the CPU.

The GPU path exchanges the plan's flat fp32 gradient buffer with one RCCL all-reduce; here the
same GradSync runs over gloo on CPU tensors (its non-plan path buckets p.grad into one flat
buffer), plus the rank-0 broadcast of parameters and BatchNorm buffers."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from yolomi import dist as ydist
        ctx = ydist.init_from_env("gloo")
        assert ctx is not None and ctx.rank == rank and ctx.world == world
        torch.manual_seed(rank)                      # ranks start from different weights
        m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8), torch.nn.Conv2d(8, 4, 1))
        with torch.no_grad():
            m[1].running_mean.fill_(float(rank + 1))
        sync = ydist.GradSync(m, ctx)
        sync.broadcast_state()
        w0 = [p.detach().clone() for p in m.parameters()]
        # per-rank gradients: rank r contributes (r + 1) * ones * index
        for i, p in enumerate(m.parameters()):
            p.grad = torch.full_like(p, float((rank + 1) * (i + 1)))
        sync.sync()
        grads = [p.grad.clone() for p in m.parameters()]
        q.put((rank, [t.tolist() for t in w0], [float(g.mean()) for g in grads],
               float(m[1].running_mean[0])))
        ydist.shutdown()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "error", repr(e), None))


def test_gradsync_world2_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in res.values():
        assert r[1] != "error", r[2]
    # parameters identical after the broadcast (rank 0's), BN buffers too
    assert res[0][1] == res[1][1]
    assert res[0][3] == res[1][3] == 1.0
    # gradients averaged: mean over ranks of (r+1)*(i+1) = 1.5*(i+1)
    for r in range(world):
        for i, g in enumerate(res[r][2]):
            assert g == pytest.approx(1.5 * (i + 1))


class _FakePlan:
    """The parts of yolomi.graph.Plan that GradSync touches: flat grads, views, the backward hook."""

    def __init__(self, model):
        self.params = [p for p in model.parameters()]
        n = sum(p.numel() for p in self.params)
        self.grad_flat = torch.zeros(n)
        self.grad_views, off = {}, 0
        for p in self.params:
            self.grad_views[id(p)] = self.grad_flat[off:off + p.numel()].view(p.shape)
            off += p.numel()
        self.grad_hook = None

    def backward(self, rank, step):
        """Write per-rank grads parameter by parameter, in reverse (as the plan's backward does)."""
        for i, p in reversed(list(enumerate(self.params))):
            self.grad_views[id(p)].fill_(float((rank + 1) * (i + 1) * (step + 1)))
            if self.grad_hook is not None:
                self.grad_hook([p])


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from yolomi import dist as ydist
        ctx = ydist.init_from_env("gloo")
        m = torch.nn.Sequential(*[torch.nn.Linear(64, 64) for _ in range(6)])
        plan = _FakePlan(m)
        m.__dict__["_ym_last_plan"] = plan
        sync = ydist.GradSync(m, ctx, bucket_mb=0.02)     # ~20 KB buckets: several per step
        res = []
        for step in range(3):                             # step 0: plain all-reduce, then buckets
            plan.backward(rank, step)
            sync.sync()
            res.append([float(plan.grad_views[id(p)].mean()) for p in plan.params])
        q.put((rank, res, len(sync.buckets.ranges)))
        ydist.shutdown()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def test_bucketed_overlap_world2_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in res.values():
        assert r[1] != "error", r[2]
    assert res[0][2] > 2                                  # the buffer really was split
    for r in range(world):
        for step, means in enumerate(res[r][1]):
            for i, g in enumerate(means):
                assert g == pytest.approx(1.5 * (i + 1) * (step + 1)), (r, step, i)
