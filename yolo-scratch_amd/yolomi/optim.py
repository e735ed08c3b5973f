"""The optimizer tail of a training step on the MI355X: clip_grad_norm_ + AdamW in three launches.

The reference ends every step with `torch.nn.utils.clip_grad_norm_(model.parameters(), 10.0)` and
`optim.AdamW(...).step()` (train_yolo11_cuda.py:58-62, 440-451).  `FusedAdamW` IS a
`torch.optim.AdamW` (same constructor, param groups, state layout and state_dict, so `last.pt`
checkpoints resume either way) whose `step()` runs csrc/optim.hip: one deterministic norm of every
gradient and one streaming AdamW pass over every parameter, the clip coefficient computed on the
device.  With `max_grad_norm` set it performs the clipping itself (`fuses_clip`); the caller then
skips clip_grad_norm_.  There is no CPU path: parameters must be fp32 CUDA tensors.
"""
from __future__ import annotations

import torch

from ._lib import AdamWEntry, YolomiError, call, lib, stream_ptr


class FusedAdamW(torch.optim.AdamW):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 max_grad_norm: float | None = None):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.max_grad_norm = max_grad_norm
        self.fuses_clip = max_grad_norm is not None
        self.last_grad_norm = None        # device scalar: what clip_grad_norm_ would have returned
        self._tables = {}
        self._partials = None

    def _table(self, entries, tag):
        """Device copy of a (p, g, m, v, offset, n) table, rebuilt when any pointer changes."""
        key = tuple(entries)
        hit = self._tables.get(tag)
        if hit is not None and hit[0] == key:
            return hit[1], hit[2], hit[3]
        arr = (AdamWEntry * len(entries))()
        off = 0
        for e, (p, g, m, v, n) in zip(arr, entries):
            e.p, e.g, e.m, e.v, e.offset, e.n = p, g, m, v, off, n
            off += n
        dev = self.param_groups[0]["params"][0].device
        t = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
        self._tables[tag] = (key, t, len(entries), off)
        return t, len(entries), off

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        groups = []
        for gi, group in enumerate(self.param_groups):
            if group["amsgrad"] or group["maximize"] or group.get("differentiable"):
                raise YolomiError("FusedAdamW: amsgrad / maximize / differentiable are not supported")
            live = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.grad.dtype == torch.float32):
                    raise YolomiError("FusedAdamW runs on the MI355X only: fp32 CUDA parameters and gradients "
                                      "(the CPU restatement lives in oracle/ and is test-only)")
                if p.grad.is_sparse or not (p.is_contiguous() and p.grad.is_contiguous()):
                    raise YolomiError("FusedAdamW: dense contiguous parameters and gradients required")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                live.append(p)
            if live:
                steps = [self.state[p]["step"] for p in live]
                torch._foreach_add_(steps, 1.0)
                groups.append((gi, group, live, steps))
        if not groups:
            return loss
        s = stream_ptr()
        norm = None
        clip = float(self.max_grad_norm) if self.max_grad_norm is not None else 0.0
        if clip > 0:
            ents = [(p.data_ptr(), p.grad.data_ptr(), 0, 0, p.numel()) for _, _, live, _ in groups for p in live]
            tab, n, total = self._table(ents, "norm")
            nb = lib().ym_grad_norm_blocks(total)
            dev = tab.device
            if self._partials is None or self._partials.numel() < nb + 1:
                self._partials = torch.empty(nb + 1, dtype=torch.float32, device=dev)
            norm = self._partials[nb:nb + 1]
            call("ym_grad_norm", tab.data_ptr(), n, total, self._partials.data_ptr(), norm.data_ptr(), s)
            self.last_grad_norm = norm
        for gi, group, live, steps in groups:
            # parameters normally share the group's step; split the launch where they do not
            by_step = {}
            for p, t in zip(live, steps):
                by_step.setdefault(int(t.item()), []).append(p)
            beta1, beta2 = group["betas"]
            lr = group["lr"]
            lr = float(lr.item()) if torch.is_tensor(lr) else float(lr)
            for k, ps in by_step.items():
                ents = []
                for p in ps:
                    st = self.state[p]
                    ents.append((p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                 st["exp_avg_sq"].data_ptr(), p.numel()))
                tab, n, total = self._table(ents, (gi, k) if len(by_step) > 1 else gi)
                call("ym_adamw", tab.data_ptr(), n, total, lr, float(beta1), float(beta2), float(group["eps"]),
                     float(group["weight_decay"]), k, clip, norm.data_ptr() if norm is not None else None, s)
        return loss
