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
        q.put((rank, res, len(sync.buckets[id(plan)].ranges)))
        ydist.shutdown()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def _trace_worker(rank, world, port, q):
    """Measurement mode (GradSync.set_trace, bench.py's dp_overlap at N > 1): every bucket's collective is recorded
    once per step, the results are unchanged, and switching it off restores the untraced launches."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from yolomi import dist as ydist
        ctx = ydist.init_from_env("gloo")
        m = torch.nn.Sequential(*[torch.nn.Linear(64, 64) for _ in range(6)])
        plan = _FakePlan(m)
        m.__dict__["_ym_last_plan"] = plan
        sync = ydist.GradSync(m, ctx, bucket_mb=0.02)
        res, traces = [], []
        for step in range(4):
            sync.set_trace(step in (1, 2))
            plan.backward(rank, step)
            sync.sync()
            traces.append([(r["bucket"], r["bytes"], r["host_done"] >= r["host_issue"]) for r in sync.last_trace()]
                          if step in (1, 2) else None)
            res.append([float(plan.grad_views[id(p)].mean()) for p in plan.params])
        b = sync.buckets[id(plan)]
        q.put((rank, res, traces, len(b.ranges), [(e - s) * 4 for s, e in b.ranges], b.trace is None))
        ydist.shutdown()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def test_bucket_trace_world2_gloo():
    res = _spawn(_trace_worker)
    for r in range(2):
        _, means, traces, nb, sizes, off = res[r]
        for step, ms in enumerate(means):
            for i, g in enumerate(ms):
                assert g == pytest.approx(1.5 * (i + 1) * (step + 1)), (r, step, i)
        for t in traces[1:3]:
            assert sorted(x[0] for x in t) == list(range(nb))           # every bucket once per step
            assert all(x[2] for x in t)
            assert sorted(x[1] for x in t) == sorted(sizes)
        assert traces[0] is None and traces[3] is None and off


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


def _spawn(target, world=2, extra=()):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q, *extra)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=180)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in res.values():
        assert r[1] != "error", r[2]
    return res


def _alternate_worker(rank, world, port, q):
    """Two plans (two batch sizes: a partial last batch) used alternately, the ADVICE r1 case: each
    plan's own hook must launch its own buckets and sync() must never reduce twice."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from yolomi import dist as ydist
        ctx = ydist.init_from_env("gloo")
        m = torch.nn.Sequential(*[torch.nn.Linear(64, 64) for _ in range(6)])
        plans = [_FakePlan(m), _FakePlan(m)]
        sync = ydist.GradSync(m, ctx, bucket_mb=0.02)
        res = []
        for step, which in enumerate((0, 1, 0, 1, 0, 0, 1, 1)):
            plan = plans[which]
            m.__dict__["_ym_last_plan"] = plan
            plan.backward(rank, step)
            sync.sync()
            res.append([float(plan.grad_views[id(p)].mean()) for p in plan.params])
        q.put((rank, res, None))
        ydist.shutdown()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def test_gradsync_alternating_plans_world2_gloo():
    res = _spawn(_alternate_worker)
    for r in range(2):
        for step, means in enumerate(res[r][1]):
            for i, g in enumerate(means):
                assert g == pytest.approx(1.5 * (i + 1) * (step + 1)), (r, step, i, g)


class _Toy(torch.utils.data.Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


def _loader_worker(rank, world, port, q, n, batch):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        import torch.distributed as dist
        from yolomi import dist as ydist
        import train_yolo11_cuda as T
        ctx = ydist.init_from_env("gloo")
        out = {}
        for epoch in range(2):
            tl, vl, sampler = T.make_loaders(_Toy(n), 0.2, batch, 0, 64, ctx, collate=lambda b: torch.tensor(b))
            sampler.set_epoch(epoch)
            steps = torch.tensor([0])
            seen = []
            for b in tl:
                steps += 1
                seen += b.tolist()
                t = torch.ones(1)
                dist.all_reduce(t)            # one collective per step, like GradSync: must never hang
            out[epoch] = (int(steps), seen, [int(i) for b in vl for i in b.tolist()])
        q.put((rank, out, None))
        ydist.shutdown()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


@pytest.mark.parametrize("n,batch", [(101, 8), (37, 4)])
def test_train_loader_equal_steps_and_val_shards_world2(n, batch):
    """make_loaders (train_yolo11_cuda.py) with an odd dataset size: every rank takes the same number of
    steps, the train shards are disjoint and reshuffled per epoch, the val shards cover the val set once."""
    res = _spawn(_loader_worker, extra=(n, batch))
    val_size = int(n * 0.2)
    for epoch in range(2):
        s0, s1 = res[0][1][epoch], res[1][1][epoch]
        assert s0[0] == s1[0] > 0
        assert not set(s0[1]) & set(s1[1])                      # disjoint train shards
        assert len(s0[1]) == len(s1[1]) == (n - val_size) // 2
        assert sorted(s0[2] + s1[2]) == sorted(set(s0[2] + s1[2])) and len(s0[2] + s1[2]) == val_size
    assert res[0][1][0][1] != res[0][1][1][1]                 # set_epoch reshuffles


def _gather_worker(rank, world, port, q, preds, targets):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from yolomi import dist as ydist
        ctx = ydist.init_from_env("gloo")
        mine = list(range(rank, len(preds), world))           # the ValShard of this rank
        gp, gt = ydist.gather_detections([preds[i] for i in mine], [targets[i] for i in mine], ctx)
        # numpy across the queue (torch tensors would travel as shared memory the exiting child owns)
        npy = (lambda L: None if L is None else [{k: v.numpy() for k, v in d.items()} for d in L])
        q.put((rank, (npy(gp), npy(gt)), None))
        ydist.shutdown()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def test_gather_detections_world2_equals_single_process():
    """Per-rank detections gathered to rank 0 reproduce the single-process list (order included), so
    evaluate_detections (oracle restatement here, CPU) gives identical metrics."""
    from oracle import metrics as omet
    g = torch.Generator().manual_seed(4)
    preds, targets = [], []
    for i in range(11):                                  # odd image count, some empty images
        k = int(torch.randint(0, 6, (1,), generator=g)) if i % 4 else 0
        t = int(torch.randint(0, 4, (1,), generator=g))
        c = torch.rand(t, 2, generator=g) * 0.8
        tb = torch.cat((c, c + 0.1 + 0.1 * torch.rand(t, 2, generator=g)), 1)
        src = tb[torch.randint(0, max(t, 1), (k,), generator=g)] if t else torch.rand(k, 4, generator=g)
        preds.append({"boxes": (src + 0.01 * torch.randn(k, 4, generator=g)).clamp(0, 1),
                      "scores": torch.rand(k, generator=g), "labels": torch.randint(0, 5, (k,), generator=g)})
        targets.append({"boxes": tb, "labels": torch.randint(0, 5, (t,), generator=g)})
    res = _spawn(_gather_worker, extra=(preds, targets))
    assert res[1][1] == (None, None)
    gp, gt = res[0][1]
    gp = [{k: torch.from_numpy(v) for k, v in d.items()} for d in gp]
    gt = [{k: torch.from_numpy(v) for k, v in d.items()} for d in gt]
    assert len(gp) == len(preds) and len(gt) == len(targets)
    for a, b in zip(gp, preds):
        for k in ("boxes", "scores", "labels"):
            assert torch.equal(a[k], b[k].reshape(a[k].shape)), k
    for a, b in zip(gt, targets):
        assert torch.equal(a["boxes"], b["boxes"]) and torch.equal(a["labels"], b["labels"])
    assert omet.evaluate_detections(gp, gt, 0.25, 0.5) == omet.evaluate_detections(preds, targets, 0.25, 0.5)
