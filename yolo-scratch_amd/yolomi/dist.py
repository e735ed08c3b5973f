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


# tools/dp_trace.sh: one tiny marker kernel on the comm stream where each bucket's collective is enqueued, so a
# kernel trace shows when the buckets go out against the backward's kernels
_MARK = os.environ.get("YM_DP_MARK") == "1"


@dataclass
class DPContext:
    rank: int
    world: int
    local_rank: int


def init_from_env(backend: str | None = None) -> DPContext | None:
    """Initialise the process group when launched by torchrun (WORLD_SIZE > 1).

    Rehearsal overrides (a multi-rank run on a one-GPU box; never set for a real DP job):
    YM_DIST_BACKEND=gloo all-reduces through the host, YM_DIST_DEVICE=0 puts every rank on GPU 0
    (RCCL refuses two ranks on one device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("YM_DIST_DEVICE") is not None:
        local = int(os.environ["YM_DIST_DEVICE"])
    backend = backend or os.environ.get("YM_DIST_BACKEND") or None
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
        self.comm = None           # the stream the bucket collectives are issued from (created on first use)
        # measurement mode (GradSync.trace; bench.py's dp_overlap at N > 1): per launched bucket, where its
        # collective starts and ends on the device (events on the comm stream, the end after the collective's
        # own stream has finished it) or on the host (gloo on CPU tensors)
        self.trace = None

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
        self.writes = [{} for _ in self.ranges]      # bucket -> {stream: event after its last write there}

    def ready(self, params, writes=None):
        """params: parameters whose gradients an op has finished; writes: the (stream, event) pairs
        recorded right after that op's gradient-writing launches (yolomi.graph.Plan.note_grad_write)."""
        for p in params:
            b = self.bucket_of.get(id(p))
            if b is None:
                continue
            for st, ev in writes or ():
                self.writes[b][st] = ev           # later writes on a stream supersede earlier ones
            self.remaining[b] -= 1
            if self.remaining[b] == 0:
                self._launch(b)

    def _launch(self, b):
        if self.trace is not None:
            return self._launch_traced(b)
        s, e = self.ranges[b]
        writes = self.writes[b] if getattr(self, "writes", None) else {}
        streams = self.streams() if self.streams else []
        if writes:
            # the collective waits for exactly the launches that wrote this bucket (the BN finalizes on
            # the scheduler's streams, the weight gradients on the side stream), on a stream of its own:
            # neither it nor the backward's streams wait for the other's unrelated work
            if self.comm is None:
                self.comm = torch.cuda.Stream(device=self.flat.device)
            for ev in writes.values():
                self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm):
                if _MARK:
                    torch.cuda._sleep(64)         # a marker kernel on the comm stream (tools/dp_trace.sh)
                self.handles.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True))
        elif len(streams) <= 1:
            self.handles.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True))
        else:
            # writers unknown: issue from the last stream after it has caught up with all the others
            comm = streams[-1]
            for o in streams[:-1]:
                comm.wait_stream(o)
            with torch.cuda.stream(comm):
                self.handles.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True))
        self.launched[b] = True

    def _launch_traced(self, b):
        """_launch with each collective bracketed: the start event after the bucket's write events (where the
        comm stream can start it), the end event after the comm stream has waited for the collective (on RCCL's
        internal stream), so end - start is the collective's wall time on the device.  The extra waits serialize
        the buckets on the comm stream, as RCCL serializes one process group's collectives anyway."""
        import time
        s, e = self.ranges[b]
        rec = {"bucket": b, "bytes": (e - s) * self.flat.element_size(), "host_issue": time.perf_counter()}
        if self.flat.is_cuda:
            if self.comm is None:
                self.comm = torch.cuda.Stream(device=self.flat.device)
            writes = self.writes[b] if getattr(self, "writes", None) else {}
            if writes:
                for ev in writes.values():
                    self.comm.wait_event(ev)
            else:
                for o in (self.streams() if self.streams else []):
                    self.comm.wait_stream(o)
                self.comm.wait_stream(torch.cuda.current_stream(self.flat.device))
            rec["start"], rec["end"] = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(self.comm):
                rec["start"].record(self.comm)
                h = dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True)
                h.wait()                          # the comm stream waits for the collective's own stream
                rec["end"].record(self.comm)
            self.handles.append(h)
        else:
            h = dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True)
            h.wait()
            rec["host_done"] = time.perf_counter()
            self.handles.append(h)
        self.trace.append(rec)
        self.launched[b] = True

    def finish(self, world: int):
        for b in range(len(self.ranges)):        # parameters no op reported (none in a full plan)
            if not self.launched[b]:
                self.writes[b] = {}
                self._launch(b)
        for h in self.handles:
            h.wait()
        self.handles = []
        self.flat.div_(world)


class GradSync:
    """Average the model's gradients across ranks; bucketed and overlapped with the backward.

    One Buckets object (and one backward hook) per plan: a model runs one plan per input shape
    (e.g. a partial last batch), and each plan's hook launches that plan's buckets only."""

    def __init__(self, model: torch.nn.Module, ctx: DPContext, bucket_mb: float = 8.0):
        self.model, self.ctx = model, ctx
        self.cap = int(bucket_mb * (1 << 20))
        self.buckets = {}          # id(plan) -> Buckets (None: plan replays a HIP graph, no hooks)
        self._plans = {}           # id(plan) -> plan (keeps the ids valid)

    def _attach(self, plan):
        """Hook the plan's backward so its NEXT backward launches buckets as it goes.  A plan that
        replays its backward as a HIP graph takes no hooks: its gradient is all-reduced in one
        collective after the backward, every step."""
        self._plans[id(plan)] = plan
        if getattr(plan, "graph_active", False):
            self.buckets[id(plan)] = None
            return
        b = Buckets(plan.grad_flat, plan.params, plan.grad_views, self.cap)
        b.streams = getattr(plan, "comm_streams", None)
        if getattr(self, "_trace_on", False):
            b.trace = []
        self.buckets[id(plan)] = b

        def hook(params, writes=None, _b=b, _plan=plan):
            if self.model.__dict__.get("_ym_pooled_step"):
                return                    # reduced after the backwards (sync), not bucket by bucket
            if not _b.remaining:
                _b.begin()
            _b.ready(params, writes)
        plan.grad_hook = hook

    def set_trace(self, on: bool):
        """Measurement mode for the following steps: every plan's buckets record their collectives (Buckets.trace);
        last_trace() returns the records of the latest step."""
        self._trace_on = on
        for b in self.buckets.values():
            if b is not None:
                b.trace = [] if on else None

    def last_trace(self):
        return list(getattr(self, "_last_trace", []))

    def sync(self):
        plan = self.model.__dict__.get("_ym_last_plan")
        tr = None
        if getattr(self, "_trace_on", False) and plan is not None:
            b = self.buckets.get(id(plan))
            tr = b.trace if b is not None else None
        try:
            self._sync(plan)
        finally:
            if tr is not None:
                self._last_trace = list(tr)
                tr.clear()

    def _sync(self, plan):
        if self.model.__dict__.pop("_ym_pooled_step", False):
            # several forwards were in flight before this step's backwards (yolomi.graph.run_model): their
            # plans' gradients were added together into .grad, which is reduced below as one buffer; the
            # flag is per step, so the next ordinary step overlaps its buckets with the backward again.
            # The decision is rank-local: a data-parallel loop must take the same forwards on every rank
            # (SPMD), as DDP requires of its own bucket hooks.
            plan = None
            for b in self.buckets.values():
                if b is not None:
                    b.remaining = []
        if plan is not None:
            b = self.buckets.get(id(plan))
            if b is not None and b.remaining:
                # this plan's backward launched its buckets: wait for them, never reduce twice
                b.finish(self.ctx.world)
                b.remaining = []           # the next backward of this plan starts a new round
                return
            # first step on this plan (or a graph-replayed backward): one collective now
            dist.all_reduce(plan.grad_flat, op=dist.ReduceOp.SUM)
            plan.grad_flat.div_(self.ctx.world)
            if id(plan) not in self.buckets:
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

    def sync_buffers(self, src: int = 0):
        """Rank 0's BatchNorm running statistics everywhere.  Each rank's BN normalises with its own
        batch statistics (plain BatchNorm2d under DDP) and updates its own running buffers; DDP's
        default broadcast_buffers=True makes rank 0's the ones that count.  Called before every
        validation and checkpoint (main), it gives every rank exactly rank 0's buffers — what DDP
        leaves on rank 0 — at the only points the running statistics are read."""
        with torch.no_grad():
            for t in self.model.buffers():
                dist.broadcast(t.data, src)


# ----------------------------------------------------------------------------- data sharding
class ValShard(torch.utils.data.Sampler):
    """Validation shard without padding: rank r takes samples r, r + world, ... in order (a
    DistributedSampler pads by repeating samples, which would count images twice in the mAP).
    gather_detections() restores the global order on rank 0."""

    def __init__(self, n: int, rank: int, world: int):
        self.n, self.rank, self.world = n, rank, world

    def __iter__(self):
        return iter(range(self.rank, self.n, self.world))

    def __len__(self):
        return len(range(self.rank, self.n, self.world))


def _pack(items, keys, widths):
    """list of per-image dicts -> (counts (n,), {key: concatenated (rows, width) blocks})"""
    counts = torch.tensor([len(it[keys[0]]) for it in items], dtype=torch.int64)
    cols = {}
    for k, w in zip(keys, widths):
        parts = [it[k].reshape(len(it[keys[0]]), w) for it in items]
        cols[k] = torch.cat(parts) if parts else None
    return counts, cols


def _all_gather_var(t: torch.Tensor, world: int):
    """all_gather of a tensor whose first dimension differs per rank (padded to the max)."""
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x) for x in ns]
    mx = max(ns)
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return [o[:k] for o, k in zip(outs, ns)]


def gather_detections(preds, targets, ctx: DPContext, device=None):
    """Per-image prediction / target dicts of every rank's ValShard -> rank 0, in the global image
    order (image i came from rank i % world, position i // world).  Non-zero ranks get (None, None).
    SURVEY §8(e): AP is not decomposable across ranks, so the matching runs on rank 0."""
    world, rank = ctx.world, ctx.rank
    dev = device or (preds[0]["boxes"].device if preds else torch.device("cpu"))
    pk = ("boxes", "scores", "labels")
    tk = ("boxes", "labels")

    def norm(items, keys):
        out = []
        for it in items:
            d = {}
            for k in keys:
                v = it[k].to(dev)
                d[k] = v.float() if k != "labels" else v.long()
            out.append(d)
        return out
    preds, targets = norm(preds, pk), norm(targets, tk)
    res = {}
    for name, items, keys in (("p", preds, pk), ("t", targets, tk)):
        widths = (4, 1, 1) if name == "p" else (4, 1)
        counts, cols = _pack(items, keys, widths)
        counts = counts.to(dev)
        g_counts = _all_gather_var(counts, world)
        g_cols = {}
        for k, w in zip(keys, widths):
            col = cols[k] if cols[k] is not None else torch.zeros(0, w, device=dev,
                                                                 dtype=torch.int64 if k == "labels" else torch.float32)
            g_cols[k] = _all_gather_var(col.reshape(-1, w), world)
        res[name] = (g_counts, g_cols, keys)
    if rank != 0:
        return None, None

    def unpack(g_counts, g_cols, keys):
        per_rank = []
        for r in range(world):
            offs = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), g_counts[r].cumsum(0)]).tolist()
            imgs = []
            for j in range(len(g_counts[r])):
                d = {}
                for k in keys:
                    v = g_cols[k][r][offs[j]:offs[j + 1]]
                    d[k] = v if k == "boxes" else v.reshape(-1)
                imgs.append(d)
            per_rank.append(imgs)
        n = sum(len(x) for x in per_rank)
        return [per_rank[i % world][i // world] for i in range(n)]
    return unpack(*res["p"]), unpack(*res["t"])
