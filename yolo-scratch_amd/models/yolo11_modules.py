"""YOLOv11 building blocks — drop-in for the reference's models/yolo11_modules.py.

Same class names, constructor signatures, attribute names and parameter
shapes as /root/reference/yolo_scratch_cuda/models/yolo11_modules.py (so
state_dict keys match and `last.pt` checkpoints interoperate).  The modules
are parameter containers: `nn.Conv2d` / `nn.BatchNorm2d` hold the fp32 master
weights and BN buffers (constructed in the reference's order, so a seeded
build draws identical initial weights), while every forward/backward runs as
libyolomi HIP kernels through the NHWC execution plan in yolomi.graph.
There is no CPU path: calling a block on a CPU tensor raises.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from yolomi.graph import run_block


def autopad(k, p=None, d=1):
    """'same' padding (reference :12-18)."""
    if d > 1:
        k = d * (k - 1) + 1 if isinstance(k, int) else [d * (x - 1) + 1 for x in k]
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


class _Block(nn.Module):
    def forward(self, x):
        return run_block(self, x)


class Conv(_Block):
    """conv(no bias) -> BatchNorm2d -> SiLU (reference :21-33)."""

    default_act = nn.SiLU()

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p, d), groups=g, dilation=d, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.act = self.default_act if act is True else act if isinstance(act, nn.Module) else nn.Identity()


class Bottleneck(_Block):
    """cv1 -> cv2 (+ x when shortcut and c1 == c2) (reference :36-47)."""

    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2


class C2f(_Block):
    """CSP bottleneck with 2 convolutions (reference :50-63)."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=(3, 3), e=1.0) for _ in range(n))


class C3k(_Block):
    """Two 1x1 branches + bottleneck chain (reference :66-78)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5, k=3):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=(k, k), e=1.0) for _ in range(n)))


class C3k2(C2f):
    """C2f with C3k or Bottleneck blocks (reference :81-89)."""

    def __init__(self, c1, c2, n=1, c3k=False, e=0.5, g=1, shortcut=True):
        super().__init__(c1, c2, n, shortcut, g, e)
        self.m = nn.ModuleList(
            C3k(self.c, self.c, 2, shortcut, g) if c3k else Bottleneck(self.c, self.c, shortcut, g, k=(3, 3), e=1.0)
            for _ in range(n))


class SPPF(_Block):
    """1x1 -> three chained 5x5 max-pools -> concat -> 1x1 (reference :92-105)."""

    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * 4, c2, 1, 1)
        self.m = nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2)
        if k != 5:
            raise NotImplementedError("SPPF pool kernel is specialised for k=5 (the only size the graph uses)")


class Attention(_Block):
    """Multi-head attention with positional dw-conv (reference :108-136).  Inside PSA it runs in PSA's
    plan; called on its own, `forward` lowers qkv 1x1 -> attention core -> + pe(v) -> proj 1x1 into a
    plan of its own (yolomi.graph._attention without the PSA residual)."""

    def __init__(self, dim, num_heads=8, attn_ratio=0.5):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.key_dim = int(self.head_dim * attn_ratio)
        self.scale = self.key_dim ** -0.5
        nh_kd = self.key_dim * num_heads
        h = dim + nh_kd * 2
        self.qkv = Conv(dim, h, 1, act=False)
        self.proj = Conv(dim, dim, 1, act=False)
        self.pe = Conv(dim, dim, 3, 1, g=dim, act=False)


class PSA(_Block):
    """b += attn(b); b += ffn(b) on half the channels (reference :139-159)."""

    def __init__(self, c1, c2, e=0.5):
        super().__init__()
        assert c1 == c2
        self.c = int(c1 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv(2 * self.c, c1, 1)
        self.attn = Attention(self.c, attn_ratio=0.5, num_heads=self.c // 64)
        self.ffn = nn.Sequential(Conv(self.c, self.c * 2, 1), Conv(self.c * 2, self.c, 1, act=False))


class C2PSA(_Block):
    """C2 block with PSA attention (reference :162-177)."""

    def __init__(self, c1, c2, n=1, e=0.5):
        super().__init__()
        assert c1 == c2
        self.c = int(c1 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv(2 * self.c, c1, 1)
        self.m = nn.Sequential(*(PSA(self.c, self.c, e=1.0) for _ in range(n)))


class DFL(nn.Module):
    """Integral of the 16-bin distribution (reference :180-192).  Its conv weight is a
    parameter of the state_dict; the eval decode kernel reads it."""

    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        x = torch.arange(c1, dtype=torch.float)
        self.conv.weight.data[:] = nn.Parameter(x.view(1, c1, 1, 1))
        self.c1 = c1

    def forward(self, x):
        """(b, 4*c1, a) -> softmax over the c1 bins of each side -> 1x1 conv with this module's weight ->
        (b, 4, a) (reference :189-192), ym_dfl_fwd; differentiable in x (ym_dfl_bwd)."""
        from yolomi.head import dfl
        return dfl(x, self.conv.weight, self.c1)


class Detect(nn.Module):
    """YOLOv8-style decoupled head (reference :195-274).  Runs inside the model's plan."""

    dynamic = False
    export = False
    end2end = False
    max_det = 300

    def __init__(self, nc=80, ch=()):
        super().__init__()
        self.nc = nc
        self.nl = len(ch)
        self.reg_max = 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.zeros(self.nl)
        self.shape = None
        c2, c3 = max((16, ch[0] // 4, self.reg_max * 4)), max(ch[0], min(self.nc, 100))
        self.cv2 = nn.ModuleList(nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * self.reg_max, 1))
                                 for x in ch)
        self.cv3 = nn.ModuleList(nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, self.nc, 1))
                                 for x in ch)
        self.dfl = DFL(self.reg_max) if self.reg_max > 1 else nn.Identity()

    def forward(self, x):
        """Train: list of (B, 64+nc, h, w) maps; eval: (y (B, 4+nc, A), maps) (reference :237-266).
        Inside a YOLOv11 the head runs as part of the model's plan; called on its own it lowers its
        six conv chains and bias convs into a plan of its own (yolomi.graph.run_detect)."""
        from yolomi.graph import run_detect
        from yolomi import head as yhead
        head, plan = run_detect(self, x)
        maps = yhead.level_views(head, plan.level_hw)
        if self.training:
            return maps
        return yhead.inference(self, head, plan.level_hw), maps

    def inference(self, x):
        """Decode a list of level maps to y (B, 4+nc, A): DFL projection with this module's weights
        (Q5), ltrb -> xywh * stride, sigmoid(cls) (reference :248-266) — ym_detect_decode."""
        from yolomi import head as yhead
        h = getattr(x[0], "_ym_head", None)
        if h is not None and all(getattr(f, "_ym_head", None) is h for f in x):
            return yhead.inference(self, h, list(x[0]._ym_levels))
        B = x[0].shape[0]
        head = torch.cat([t.reshape(B, self.no, -1) for t in x], 2).permute(0, 2, 1).float().contiguous()
        return yhead.inference(self, head, [tuple(t.shape[2:]) for t in x])

    def bias_init(self):
        """Reference :268-274; called while stride is still zero."""
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            s = float(s)
            ratio = math.inf if s == 0 else 640 / s
            bias_value = 5 / self.nc / max(ratio ** 2, 1.0)
            b[-1].bias.data[: self.nc] = math.log(max(bias_value, 1e-6))


class Concat(nn.Module):
    """Channel concatenation (reference :277-285); a buffer-slice plan inside the model."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def forward(self, x):
        """torch.cat(x, self.d) (reference :284-285).  Inside a YOLOv11 a concat is free (producers
        write channel slices of one buffer); called on its own it is a strided device copy per input
        (ym_copy2d), differentiable."""
        from yolomi.concat import concat
        return concat(list(x), self.d)


def make_anchors(feats, strides, grid_cell_offset=0.5):
    """Anchor centres and strides per level (reference :288-300); a tiny host-side table."""
    anchor_points, stride_tensor = [], []
    dtype, device = feats[0].dtype, feats[0].device
    for i, stride in enumerate(strides):
        _, _, h, w = feats[i].shape
        sx = torch.arange(end=w, device=device, dtype=dtype) + grid_cell_offset
        sy = torch.arange(end=h, device=device, dtype=dtype) + grid_cell_offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        anchor_points.append(torch.stack((sx, sy), -1).view(-1, 2))
        stride_tensor.append(torch.full((h * w, 1), float(stride), dtype=dtype, device=device))
    return torch.cat(anchor_points), torch.cat(stride_tensor)


def dist2bbox(distance, anchor_points, xywh=True, dim=-1):
    """ltrb distances -> xywh / xyxy boxes (reference :303-312)."""
    lt, rb = distance.chunk(2, dim)
    x1y1 = anchor_points - lt
    x2y2 = anchor_points + rb
    if xywh:
        return torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), dim)
    return torch.cat((x1y1, x2y2), dim)
