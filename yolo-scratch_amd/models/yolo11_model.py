"""YOLOv11 model built from the YAML graph — drop-in for the reference's models/yolo11_model.py.

Graph parse, weight init and Detect stride bookkeeping follow
/root/reference/yolo_scratch_cuda/models/yolo11_model.py (YOLOv11 :17-252,
build_yolo11 :258-288) so layer indices, `save`, channel widths and the
state_dict are identical; the quirks the reference's construction leaves in
the weights are reproduced.  Two differences in HOW:
the module names in the YAML are resolved through an explicit registry (no
eval), and Detect.stride is derived from the graph's strides instead of a
dummy 640x640 CPU forward — the BN buffers are set to exactly the values that
forward leaves behind (mean 0, var 0.97, num_batches_tracked 1, Q6).

forward(x) runs the whole network as one NHWC plan of HIP kernels
(yolomi.graph).  Train mode returns the list of three (B, 64+nc, H, W) head
maps — views into one (B, A, 64+nc) fp32 buffer; eval mode returns
(y (B, 4+nc, A), maps) like Detect.inference (yolo11_modules.py:248-266).
"""
from __future__ import annotations

import contextlib
import io
import math
from pathlib import Path

import torch
import torch.nn as nn
import yaml

from .yolo11_modules import C2PSA, C3k2, SPPF, Bottleneck, C2f, Concat, Conv, Detect, DFL  # noqa: F401

_REGISTRY = {"Conv": Conv, "C3k2": C3k2, "C2PSA": C2PSA, "SPPF": SPPF, "Bottleneck": Bottleneck, "C2f": C2f,
             "Concat": Concat, "Detect": Detect, "nn.Upsample": nn.Upsample, "Upsample": nn.Upsample,
             "nn.BatchNorm2d": nn.BatchNorm2d}


class YOLOv11(nn.Module):
    def __init__(self, cfg="configs/yolo11n_crater.yaml", ch=1, nc=5, verbose=True):
        super().__init__()
        if isinstance(cfg, dict):
            self.yaml = cfg
        else:
            with open(cfg) as f:
                self.yaml = yaml.safe_load(f)
        self.yaml["ch"] = ch
        self.yaml["nc"] = nc
        self.model, self.save = self.parse_model(self.yaml, ch, verbose)
        self.names = [str(i) for i in range(nc)]
        self.inplace = True
        self._initialize_weights()
        self._compute_strides()

    # ------------------------------------------------------------------ forward
    def forward(self, x):
        return self._forward_once(x)

    def _forward_once(self, x):
        from yolomi.graph import run_model
        from yolomi import head as yhead
        head, plan = run_model(self, x)
        maps = yhead.level_views(head, plan.level_hw)
        if self.training:
            return maps
        return yhead.inference(self.model[-1], head, plan.level_hw), maps

    # ------------------------------------------------------------------ construction
    def parse_model(self, d, ch, verbose=True):
        """YAML -> nn.Sequential (reference :73-170)."""
        scale = d.get("scale")
        if scale is None or scale not in d["scales"]:
            scale = list(d["scales"].keys())[0]
        nc, gd, gw = d["nc"], d["scales"][scale][0], d["scales"][scale][1]
        if verbose:
            print(f"Using scale '{scale}': depth={gd}, width={gw}")
        ch = [ch] if isinstance(ch, int) else ch
        layers, save, c2 = [], [], ch[-1]
        self._layer_stride = []
        for i, (f, n, m, args) in enumerate(d["backbone"] + d["head"]):
            m = _REGISTRY[m] if isinstance(m, str) else m
            args = list(args)
            for j, a in enumerate(args):
                if isinstance(a, str):
                    args[j] = {"nc": nc, "None": None}.get(a, a)
            n = max(round(n * gd), 1) if n > 1 else n
            if m in (Conv, Bottleneck, SPPF, C2f, C3k2, C2PSA):
                c1, c2 = ch[f], args[0]
                if c2 != nc:
                    c2 = self.make_divisible(c2 * gw, 8)
                args = [c1, c2, *args[1:]]
                if m in (C2f, C3k2, C2PSA):
                    args.insert(2, n)
                    n = 1
            elif m is nn.BatchNorm2d:
                args = [ch[f]]
            elif m is Concat:
                c2 = sum(ch[x] for x in f)
            elif m is Detect:
                args.append([ch[x] for x in f])
            else:
                c2 = ch[f]
            m_ = nn.Sequential(*(m(*args) for _ in range(n))) if n > 1 else m(*args)
            m_.i, m_.f, m_.type = i, f, m.__name__
            # stride bookkeeping for Detect (replaces the dummy-forward probe)
            prev = self._layer_stride
            src = (prev[f] if f != -1 else (prev[-1] if prev else 1)) if isinstance(f, int) else None
            if m is Conv:
                st = src * m_.conv.stride[0]
            elif m is nn.Upsample:
                st = src / 2
            elif m is Concat:
                st = prev[f[0]] if f[0] != -1 else prev[-1]
            elif m is Detect:
                st = [prev[x] for x in f]
            else:
                st = src
            self._layer_stride.append(st)
            if verbose:
                npar = sum(x.numel() for x in m_.parameters())
                print(f"{i:>3}{str(f):>20}{n:>3}{npar:>10}  {m_.type:<20}{str(args):<30}")
            save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
            layers.append(m_)
            if i == 0:
                ch = []
            ch.append(c2)
        return nn.Sequential(*layers), sorted(save)

    @staticmethod
    def make_divisible(x, divisor=8):
        return math.ceil(x / divisor) * divisor

    def _initialize_weights(self):
        """Reference :177-192: kaiming fan_out on every Conv2d (DFL included, Q5), BN eps/momentum, bias_init."""
        for m in self.modules():
            t = type(m)
            if t is nn.Conv2d:
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif t is nn.BatchNorm2d:
                m.eps = 1e-3
                m.momentum = 0.03
            elif t in (nn.Hardswish, nn.LeakyReLU, nn.ReLU, nn.ReLU6, nn.SiLU):
                m.inplace = True
        for m in self.modules():
            if hasattr(m, "bias_init"):
                m.bias_init()

    def _compute_strides(self):
        """Detect.stride from the graph; BN buffers as the reference's zero-image probe leaves them (Q6, Q7)."""
        det = self.model[-1]
        if not isinstance(det, Detect):
            return
        det.stride = torch.tensor([float(s) for s in self._layer_stride[-1]], dtype=torch.float32)
        with torch.no_grad():
            for m in self.modules():
                if isinstance(m, nn.BatchNorm2d):
                    m.running_mean.zero_()
                    m.running_var.fill_(0.97)
                    m.num_batches_tracked.fill_(1)

    def info(self, verbose=False, img_size=640):
        n_p = sum(x.numel() for x in self.parameters())
        n_g = sum(x.numel() for x in self.parameters() if x.requires_grad)
        print(f"Model Summary: {len(list(self.modules()))} layers, {n_p} parameters, {n_g} gradients")


def build_yolo11(cfg="configs/yolo11n_crater.yaml", ch=1, nc=5, pretrained=None):
    """Reference :258-288 (local checkpoint loading only; weights_only=True)."""
    if isinstance(cfg, (str, Path)) and not Path(cfg).exists():
        alt = Path(__file__).resolve().parents[1] / cfg
        if alt.exists():
            cfg = str(alt)
    with contextlib.redirect_stdout(io.StringIO()):
        model = YOLOv11(cfg=cfg, ch=ch, nc=nc)
    if pretrained:
        ckpt = torch.load(pretrained, map_location="cpu", weights_only=True)
        state = ckpt.get("model", ckpt.get("model_state_dict", ckpt)) if isinstance(ckpt, dict) else ckpt
        model.load_state_dict(state, strict=False)
    return model
