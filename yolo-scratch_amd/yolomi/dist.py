"""Data parallelism: one process per GPU, RCCL (torch.distributed 'nccl') over xGMI.

The reference is single-process; this is the build's DP layer for
BASELINE configs C3 (8 x MI355X).  Each rank runs the whole YOLOv11 plan on its
own minibatch (BatchNorm keeps per-rank batch statistics, as plain BatchNorm2d
under DDP would).  Parameter gradients live in ONE flat fp32 buffer per plan
(yolomi.graph.Plan.grad_flat) so the exchange is a single all-reduce, issued on
RCCL's stream right after the backward, followed by clip_grad_norm_ and AdamW
on identical averaged gradients.
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


class GradSync:
    """Average the model's gradients across ranks with one collective per step."""

    def __init__(self, model: torch.nn.Module, ctx: DPContext):
        self.model, self.ctx = model, ctx

    def _flat(self):
        plan = self.model.__dict__.get("_ym_last_plan")
        if plan is not None:
            return plan.grad_flat
        return None

    def sync(self):
        flat = self._flat()
        if flat is not None:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM)
            flat.div_(self.ctx.world)
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
