"""Functional fp32 CPU restatement of the YOLOv11 graph — TEST ORACLE ONLY.

Every function cites the reference code it restates
(/root/reference/yolo_scratch_cuda/...).  Parameters live in a flat dict that
uses the reference's state_dict key names, so the same dict loads into the
product model.  Backward is plain CPU autograd over these fp32 ops.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

BN_EPS, BN_MOM = 1e-3, 0.03          # yolo11_model.py:183-185


# ----------------------------------------------------------------------------- graph parse
def _div8(x):                        # make_divisible, yolo11_model.py:172-175
    return math.ceil(x / 8) * 8


def parse(cfg: dict, ch: int = 1, nc: int = 5):
    """Restates YOLOv11.parse_model (yolo11_model.py:73-170).

    Returns (layers, save) where each layer is a dict with keys
    i, f, type, and the constructor arguments the reference would pass.
    """
    scale = cfg.get("scale")
    if scale is None or scale not in cfg["scales"]:
        scale = list(cfg["scales"].keys())[0]                # :91-93
    gd, gw = cfg["scales"][scale][0], cfg["scales"][scale][1]   # max_channels ignored (:98)
    chs = [ch]
    layers, save = [], []
    for i, (f, n, m, args) in enumerate(cfg["backbone"] + cfg["head"]):
        args = list(args)
        n = max(round(n * gd), 1) if n > 1 else n               # :121
        L = {"i": i, "f": f, "type": m}
        if m in ("Conv", "C3k2", "SPPF", "C2PSA"):
            c1, c2 = chs[f], args[0]
            if c2 != nc:
                c2 = _div8(c2 * gw)                             # :124-126
            L.update(c1=c1, c2=c2)
            if m == "Conv":
                L.update(k=args[1] if len(args) > 1 else 1, s=args[2] if len(args) > 2 else 1)
            elif m == "C3k2":
                L.update(n=n, c3k=bool(args[1]) if len(args) > 1 else False,
                         e=float(args[2]) if len(args) > 2 else 0.5)
            elif m == "SPPF":
                L.update(k=args[1] if len(args) > 1 else 5)
            else:
                L.update(n=n)
        elif m == "Concat":
            c2 = sum(chs[x] for x in f)
        elif m == "Detect":
            c2 = None
            L.update(nc=nc, ch=[chs[x] for x in f])
        else:                                                   # nn.Upsample
            c2 = chs[f]
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(L)
        if i == 0:
            chs = []
        chs.append(c2)
    return layers, sorted(save)


# ----------------------------------------------------------------------------- parameters
def _conv_keys(P, pre, c1, c2, k, g=1):
    P[pre + ".conv.weight"] = torch.empty(c2, c1 // g, k, k)
    P[pre + ".bn.weight"] = torch.ones(c2)
    P[pre + ".bn.bias"] = torch.zeros(c2)
    P[pre + ".bn.running_mean"] = torch.zeros(c2)
    P[pre + ".bn.running_var"] = torch.full((c2,), 0.97)       # Q6: after the stride probe
    P[pre + ".bn.num_batches_tracked"] = torch.tensor(1)


def _bottleneck_keys(P, pre, c1, c2, e=1.0):
    c_ = int(c2 * e)
    _conv_keys(P, pre + ".cv1", c1, c_, 3)
    _conv_keys(P, pre + ".cv2", c_, c2, 3)


def _c3k_keys(P, pre, c1, c2, n=2, e=0.5):
    c_ = int(c2 * e)
    _conv_keys(P, pre + ".cv1", c1, c_, 1)
    _conv_keys(P, pre + ".cv2", c1, c_, 1)
    _conv_keys(P, pre + ".cv3", 2 * c_, c2, 1)
    for j in range(n):
        _bottleneck_keys(P, f"{pre}.m.{j}", c_, c_)


def init_params(layers) -> dict:
    """Parameter/buffer dict with reference key names (random weights filled by caller)."""
    P = {}
    for L in layers:
        pre, t = f"model.{L['i']}", L["type"]
        if t == "Conv":
            _conv_keys(P, pre, L["c1"], L["c2"], L["k"])
        elif t == "C3k2":
            c = int(L["c2"] * L["e"])
            _conv_keys(P, pre + ".cv1", L["c1"], 2 * c, 1)
            _conv_keys(P, pre + ".cv2", (2 + L["n"]) * c, L["c2"], 1)
            for j in range(L["n"]):
                if L["c3k"]:
                    _c3k_keys(P, f"{pre}.m.{j}", c, c)
                else:
                    _bottleneck_keys(P, f"{pre}.m.{j}", c, c)
        elif t == "SPPF":
            c_ = L["c1"] // 2
            _conv_keys(P, pre + ".cv1", L["c1"], c_, 1)
            _conv_keys(P, pre + ".cv2", c_ * 4, L["c2"], 1)
        elif t == "C2PSA":
            c = int(L["c1"] * 0.5)
            _conv_keys(P, pre + ".cv1", L["c1"], 2 * c, 1)
            _conv_keys(P, pre + ".cv2", 2 * c, L["c1"], 1)
            for j in range(L["n"]):
                q = f"{pre}.m.{j}"
                _conv_keys(P, q + ".cv1", c, 2 * c, 1)
                _conv_keys(P, q + ".cv2", 2 * c, c, 1)
                heads = c // 64
                kd = (c // heads) // 2
                _conv_keys(P, q + ".attn.qkv", c, c + 2 * kd * heads, 1)
                _conv_keys(P, q + ".attn.proj", c, c, 1)
                _conv_keys(P, q + ".attn.pe", c, c, 3, g=c)
                _conv_keys(P, q + ".ffn.0", c, 2 * c, 1)
                _conv_keys(P, q + ".ffn.1", 2 * c, c, 1)
        elif t == "Detect":
            ch, nc = L["ch"], L["nc"]
            c2, c3 = max(16, ch[0] // 4, 64), max(ch[0], min(nc, 100))   # yolo11_modules.py:219
            for li, x in enumerate(ch):
                _conv_keys(P, f"{pre}.cv2.{li}.0", x, c2, 3)
                _conv_keys(P, f"{pre}.cv2.{li}.1", c2, c2, 3)
                P[f"{pre}.cv2.{li}.2.weight"] = torch.empty(64, c2, 1, 1)
                P[f"{pre}.cv2.{li}.2.bias"] = torch.ones(64)            # Q4 box bias
            for li, x in enumerate(ch):
                _conv_keys(P, f"{pre}.cv3.{li}.0", x, c3, 3)
                _conv_keys(P, f"{pre}.cv3.{li}.1", c3, c3, 3)
                P[f"{pre}.cv3.{li}.2.weight"] = torch.empty(nc, c3, 1, 1)
                P[f"{pre}.cv3.{li}.2.bias"] = torch.full((nc,), math.log(1e-6))   # Q4
            P[f"{pre}.dfl.conv.weight"] = torch.empty(1, 16, 1, 1)
    return P


# ----------------------------------------------------------------------------- forward
def conv(P, pre, x, s=1, act=True, training=True):
    """Conv = conv2d(no bias, p=k//2) -> BatchNorm2d -> SiLU (yolo11_modules.py:21-33)."""
    w = P[pre + ".conv.weight"]
    g = x.shape[1] // w.shape[1]
    y = F.conv2d(x, w, None, s, w.shape[-1] // 2, 1, g)
    rm, rv = P[pre + ".bn.running_mean"], P[pre + ".bn.running_var"]
    y = F.batch_norm(y, rm, rv, P[pre + ".bn.weight"], P[pre + ".bn.bias"], training, BN_MOM, BN_EPS)
    if training:
        P[pre + ".bn.num_batches_tracked"] += 1
    return F.silu(y) if act else y


def bottleneck(P, pre, x, shortcut=True, tr=True):      # yolo11_modules.py:36-47
    y = conv(P, pre + ".cv2", conv(P, pre + ".cv1", x, training=tr), training=tr)
    return x + y if (shortcut and x.shape[1] == y.shape[1]) else y


def c3k(P, pre, x, n=2, tr=True):                       # yolo11_modules.py:66-78
    a = conv(P, pre + ".cv1", x, training=tr)
    for j in range(n):
        a = bottleneck(P, f"{pre}.m.{j}", a, True, tr)
    return conv(P, pre + ".cv3", torch.cat((a, conv(P, pre + ".cv2", x, training=tr)), 1), training=tr)


def c3k2(P, pre, x, n, c3k_flag, tr=True):              # C2f.forward :59-63 with C3k2 blocks :81-89
    y = conv(P, pre + ".cv1", x, training=tr)
    c = y.shape[1] // 2
    ys = [y[:, :c], y[:, c:]]
    for j in range(n):
        ys.append(c3k(P, f"{pre}.m.{j}", ys[-1], 2, tr) if c3k_flag else bottleneck(P, f"{pre}.m.{j}", ys[-1], True, tr))
    return conv(P, pre + ".cv2", torch.cat(ys, 1), training=tr)


def sppf(P, pre, x, k=5, tr=True):                      # yolo11_modules.py:92-105
    ys = [conv(P, pre + ".cv1", x, training=tr)]
    for _ in range(3):
        ys.append(F.max_pool2d(ys[-1], k, 1, k // 2))
    return conv(P, pre + ".cv2", torch.cat(ys, 1), training=tr)


def attention(P, pre, x, tr=True):                      # yolo11_modules.py:108-136
    B, C, H, W = x.shape
    N = H * W
    heads = C // 64
    hd = C // heads
    kd = hd // 2
    qkv = conv(P, pre + ".qkv", x, act=False, training=tr)
    q, k, v = qkv.view(B, heads, 2 * kd + hd, N).split([kd, kd, hd], 2)
    a = (q.transpose(-2, -1) @ k) * (kd ** -0.5)
    a = a.softmax(-1)
    o = (v @ a.transpose(-2, -1)).view(B, C, H, W) + conv(P, pre + ".pe", v.reshape(B, C, H, W), act=False, training=tr)
    return conv(P, pre + ".proj", o, act=False, training=tr)


def psa(P, pre, x, tr=True):                            # yolo11_modules.py:139-159
    y = conv(P, pre + ".cv1", x, training=tr)
    c = y.shape[1] // 2
    a, b = y[:, :c], y[:, c:]
    b = b + attention(P, pre + ".attn", b, tr)
    b = b + conv(P, pre + ".ffn.1", conv(P, pre + ".ffn.0", b, training=tr), act=False, training=tr)
    return conv(P, pre + ".cv2", torch.cat((a, b), 1), training=tr)


def c2psa(P, pre, x, n, tr=True):                       # yolo11_modules.py:162-177
    y = conv(P, pre + ".cv1", x, training=tr)
    c = y.shape[1] // 2
    a, b = y[:, :c], y[:, c:]
    for j in range(n):
        b = psa(P, f"{pre}.m.{j}", b, tr)
    return conv(P, pre + ".cv2", torch.cat((a, b), 1), training=tr)


def anchors(shapes, strides, offset=0.5):
    """make_anchors (yolo_v8_loss.py:541-552 / yolo11_modules.py:288-300), fp32."""
    pts, st = [], []
    for (h, w), s in zip(shapes, strides):
        sx = torch.arange(w, dtype=torch.float32) + offset
        sy = torch.arange(h, dtype=torch.float32) + offset
        yy, xx = torch.meshgrid(sy, sx, indexing="ij")
        pts.append(torch.stack((xx, yy), -1).view(-1, 2))
        st.append(torch.full((h * w, 1), float(s)))
    return torch.cat(pts), torch.cat(st)


def detect(P, pre, xs, nc, strides, tr=True):           # yolo11_modules.py:237-266
    outs = []
    for li, x in enumerate(xs):
        bx = conv(P, f"{pre}.cv2.{li}.1", conv(P, f"{pre}.cv2.{li}.0", x, training=tr), training=tr)
        bx = F.conv2d(bx, P[f"{pre}.cv2.{li}.2.weight"], P[f"{pre}.cv2.{li}.2.bias"])
        cl = conv(P, f"{pre}.cv3.{li}.1", conv(P, f"{pre}.cv3.{li}.0", x, training=tr), training=tr)
        cl = F.conv2d(cl, P[f"{pre}.cv3.{li}.2.weight"], P[f"{pre}.cv3.{li}.2.bias"])
        outs.append(torch.cat((bx, cl), 1))
    if tr:
        return outs
    return inference(P, pre, outs, nc, strides), outs


def inference(P, pre, outs, nc, strides):
    """Detect.inference (yolo11_modules.py:248-266) incl. the DFL 1x1 conv (Q5)."""
    B = outs[0].shape[0]
    no = nc + 64
    xc = torch.cat([o.view(B, no, -1) for o in outs], 2)
    anc, st = anchors([o.shape[2:] for o in outs], strides)
    box, cls = xc.split((64, nc), 1)
    A = box.shape[-1]
    p = box.view(B, 4, 16, A).transpose(2, 1).softmax(1)               # DFL :190-192
    d = F.conv2d(p, P[f"{pre}.dfl.conv.weight"]).view(B, 4, A)
    lt, rb = d.chunk(2, 1)
    a = anc.t().unsqueeze(0)
    x1y1, x2y2 = a - lt, a + rb
    dbox = torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), 1) * st.t()
    return torch.cat((dbox, cls.sigmoid()), 1)


def forward(P, layers, save, x, training=True, strides=(8.0, 16.0, 32.0), keep_all=None):
    """YOLOv11._forward_once (yolo11_model.py:60-71).  keep_all: optional list receiving every layer output."""
    ys = []
    for L in layers:
        f, t, pre = L["f"], L["type"], f"model.{L['i']}"
        if f != -1:
            x = ys[f] if isinstance(f, int) else [x if j == -1 else ys[j] for j in f]
        if t == "Conv":
            x = conv(P, pre, x, L["s"], training=training)
        elif t == "C3k2":
            x = c3k2(P, pre, x, L["n"], L["c3k"], training)
        elif t == "SPPF":
            x = sppf(P, pre, x, L["k"], training)
        elif t == "C2PSA":
            x = c2psa(P, pre, x, L["n"], training)
        elif t == "Concat":
            x = torch.cat(x, 1)
        elif t == "Detect":
            x = detect(P, pre, x, L["nc"], strides, training)
        else:
            x = F.interpolate(x, scale_factor=2.0, mode="nearest")
        ys.append(x if L["i"] in save else None)
        if keep_all is not None:
            keep_all.append(x)
    return x


def build(cfg: dict, ch: int = 1, nc: int = 5, seeded: bool = True):
    from .weights import apply_seeded_weights
    layers, save = parse(cfg, ch, nc)
    P = init_params(layers)
    if seeded:
        apply_seeded_weights(P)
    return layers, save, P


def block_params(layer: dict, prefix: str = "blk", seeded: bool = True) -> dict:
    """Parameters of ONE building block (layer dict as parse() makes it, e.g. {"type": "C2PSA",
    "c1": 512, "c2": 512, "n": 1}) under `prefix.`, key-seeded as the standalone module's
    state_dict would be (oracle/weights.py)."""
    from .weights import apply_seeded_weights
    P = init_params([{**layer, "i": 0}])
    P = {prefix + k[len("model.0"):]: v for k, v in P.items()}
    if seeded:
        apply_seeded_weights(P, prefix + ".")
    return P


def load_cfg(scale: str) -> dict:
    import yaml
    from pathlib import Path
    p = Path(__file__).resolve().parents[1] / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml"
    d = yaml.safe_load(p.read_text())
    d["scale"] = scale
    return d
