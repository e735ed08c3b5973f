"""Data parallelism: one process per GPU, RCCL (torch.distributed 'nccl') over xGMI.

The reference is single-process; this is the build's DP layer for
BASELINE configs C3 (8 x MI355X).  Each rank runs the whole YOLOv11 plan on its
own minibatch (BatchNorm keeps per-rank batch statistics, as plain BatchNorm2d
under DDP would).  Parameter gradients live in ONE flat fp32 buffer per plan
(yolomi.graph.Plan.grad_flat).  The buffer is cut into ~8 MB buckets along parameter
boundaries; the plan's backward reports each op's finished parameters, and a bucket's
all-reduce is issued (async, on RCCL's stream, ordered after the kernels that wrote it) as
soon as its last parameter is done — backward runs head -> stem, so the late buckets of the
buffer go out while the backbone's dgrad/wgrad kernels still run.  sync() waits for the
buckets, averages, and the step continues with clip_grad_norm_ and AdamW on identical
gradients.  Bucket size: 45.5 MB of gradients (s) over a ring of 8 is 7/8 x 2 x 45.5 MB per
rank; 8 MB buckets keep 6 collectives in flight without making each one latency-bound.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DPContext:
    rank: int
    world: int
    local_rank: int


def init_from_env(backend: str | None = None) -> DPContext | None:
    """Initialise the process group when launched by torchrun (WORLD_SIZE > 1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return DPContext(rank, world, local)


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()


class Buckets:
    """Contiguous ranges of a flat gradient buffer, all-reduced as their parameters finish."""

    def __init__(self, flat: torch.Tensor, params, views: dict, cap_bytes: int = 8 << 20):
        self.flat = flat
        spans = sorted((views[id(p)].data_ptr(), views[id(p)].numel(), id(p)) for p in params)
        base = flat.data_ptr()
        esz = flat.element_size()
        self.ranges, self.members, self.bucket_of = [], [], {}
        cur, start, size = [], None, 0
        for ptr, n, pid in spans:
            off = (ptr - base) // esz
            if start is None:
                start = off
            cur.append(pid)
            size = off + n - start
            if size * esz >= cap_bytes:
                self._close(start, size, cur)
                cur, start, size = [], None, 0
        if cur:
            self._close(start, size, cur)
        self.handles = []
        self.remaining = []
        self.streams = None        # callable -> the producing plan's streams (yolomi.graph.Plan.comm_streams)

    def _close(self, start, size, members):
        b = len(self.ranges)
        self.ranges.append((start, start + size))
        self.members.append(members)
        for pid in members:
            self.bucket_of[pid] = b

    def begin(self):
        self.remaining = [len(m) for m in self.members]
        self.launched = [False] * len(self.ranges)
        self.handles = []

    def ready(self, params):
        for p in params:
            b = self.bucket_of.get(id(p))
            if b is None:
                continue
            self.remaining[b] -= 1
            if self.remaining[b] == 0:
                self._launch(b)

    def _launch(self, b):
        s, e = self.ranges[b]
        streams = self.streams() if self.streams else []
        if len(streams) <= 1:
            self.handles.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True))
        else:
            # the bucket's gradients come from several streams (BN backward on the scheduler's
            # streams, weight gradients on the side stream): the collective is issued from the last
            # of them after it has caught up with the others, so RCCL orders it after all writers
            comm = streams[-1]
            for o in streams[:-1]:
                comm.wait_stream(o)
            with torch.cuda.stream(comm):
                self.handles.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True))
        self.launched[b] = True

    def finish(self, world: int):
        for b in range(len(self.ranges)):        # parameters no op reported (none in a full plan)
            if not self.launched[b]:
                self._launch(b)
        for h in self.handles:
            h.wait()
        self.handles = []
        self.flat.div_(world)


class GradSync:
    """Average the model's gradients across ranks; bucketed and overlapped with the backward."""

    def __init__(self, model: torch.nn.Module, ctx: DPContext, bucket_mb: float = 8.0):
        self.model, self.ctx = model, ctx
        self.cap = int(bucket_mb * (1 << 20))
        self.plan, self.buckets = None, None

    def _attach(self, plan):
        """Hook the plan's backward so the NEXT backward launches buckets as it goes.  A plan that
        replays its backward as a HIP graph takes no hooks: its gradient is all-reduced in one
        collective after the backward (sync's first-step path, every step)."""
        if getattr(plan, "graph_active", False):
            return
        self.plan = plan
        self.buckets = Buckets(plan.grad_flat, plan.params, plan.grad_views, self.cap)
        self.buckets.streams = getattr(plan, "comm_streams", None)

        def hook(params, _b=self.buckets):
            if not _b.remaining:
                _b.begin()
            _b.ready(params)
        plan.grad_hook = hook

    def sync(self):
        plan = self.model.__dict__.get("_ym_last_plan")
        if plan is not None:
            if plan is self.plan and self.buckets.remaining:
                self.buckets.finish(self.ctx.world)
                self.buckets.remaining = []       # the next backward starts a new round
                return
            # first step on this plan: one collective now, buckets from the next step on
            dist.all_reduce(plan.grad_flat, op=dist.ReduceOp.SUM)
            plan.grad_flat.div_(self.ctx.world)
            self._attach(plan)
            return
        # gradients not produced by a yolomi plan (CPU / gloo tests): bucket them in one flat tensor
        grads = [p.grad for p in self.model.parameters() if p.grad is not None]
        if not grads:
            return
        buf = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        buf.div_(self.ctx.world)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(buf[off:off + n].view_as(g))
            off += n

    def broadcast_state(self, src: int = 0):
        """Rank 0's parameters and BN buffers everywhere (DDP's initial sync)."""
        with torch.no_grad():
            for t in list(self.model.parameters()) + list(self.model.buffers()):
                dist.broadcast(t.data, src)
