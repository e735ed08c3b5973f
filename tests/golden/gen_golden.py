#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE.

This script is the only place that imports /root/reference (read-only,
PYTHONDONTWRITEBYTECODE=1).  It runs in the development container only; the
fixtures it writes (inputs + expected outputs, .npz / .json) are committed and
travel to the GPU box, the reference never does.

Re-run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

`cv2` (OpenCV) is not installed here; the reference's train script imports it
only for image loading (datasets/crater_dataset_cuda.py:20), so a stub module
is inserted before importing `train_yolo11_cuda`.
"""
from __future__ import annotations

import copy
import importlib.util
import json
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path("/root/reference/yolo_scratch_cuda")

sys.path.insert(0, str(REPO))
from oracle.weights import apply_seeded_weights  # noqa: E402

sys.modules.setdefault("cv2", types.ModuleType("cv2"))
sys.path.insert(0, str(REF))
import train_yolo11_cuda as ref_train  # noqa: E402
from losses.yolo_v8_loss import v8DetectionLoss  # noqa: E402
from models.yolo11_model import build_yolo11  # noqa: E402
from utils.metrics import evaluate_detections  # noqa: E402
import models.yolo11_modules as ref_mods  # noqa: E402
import losses.yolo_v8_loss as ref_loss_mod  # noqa: E402
import yaml  # noqa: E402


def _load_synth():
    p = REPO / "yolo-scratch_amd" / "datasets" / "synthetic.py"
    spec = importlib.util.spec_from_file_location("ym_synthetic", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


synth = _load_synth()
torch.set_num_threads(os.cpu_count())


def cfg(scale: str) -> dict:
    with open(REF / "configs" / "yolo11n_crater.yaml") as f:
        d = yaml.safe_load(f)
    d["scale"] = scale
    return d


def build(scale: str):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        m = build_yolo11(cfg=cfg(scale), ch=1, nc=5)
    apply_seeded_weights(m.state_dict())
    return m


def save(name: str, **arrs):
    out = {}
    for k, v in arrs.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        out[k] = np.asarray(v)
    np.savez_compressed(HERE / name, **out)
    print(f"wrote {name}: {sum(a.nbytes for a in out.values()) / 1e6:.2f} MB raw, {len(out)} arrays")


# --------------------------------------------------------------------------- structure
def gen_structure():
    info = {}
    for scale in ("n", "s", "m"):
        m = build(scale)
        sd = m.state_dict()
        info[scale] = {
            "keys": [[k, list(v.shape), str(v.dtype)] for k, v in sd.items()],
            "n_params": int(sum(p.numel() for p in m.parameters())),
            "save": list(m.save),
            "stride": m.model[-1].stride.tolist(),
            "bn_running_var": float(sd["model.0.bn.running_var"][0]),
            "bn_nbt": int(sd["model.0.bn.num_batches_tracked"]),
            "detect_bias_cls": float(sd["model.23.cv3.0.2.bias"][0]),
            "detect_bias_box": float(sd["model.23.cv2.0.2.bias"][0]),
        }
    (HERE / "structure.json").write_text(json.dumps(info))
    print("wrote structure.json")


# --------------------------------------------------------------------------- NMS / IoU
def gen_nms():
    arrs = {}
    preds = synth.synth_eval_preds(1, 8400, seed=11)[0]
    xywh, sc = preds[:, :4], preds[:, 4:].max(1).values
    x1y1 = xywh[:, :2] - xywh[:, 2:] / 2
    x2y2 = xywh[:, :2] + xywh[:, 2:] / 2
    allb = torch.cat((x1y1, x2y2), 1)
    for n in (0, 1, 2, 100, 1000, 6700):
        b, s = allb[:n].contiguous(), sc[:n].contiguous()
        keep = ref_train.nms_simple(b, s, 0.45)
        arrs[f"n{n}_boxes"], arrs[f"n{n}_scores"] = b, s
        arrs[f"n{n}_keep"] = np.asarray(keep, dtype=np.int64)
    # IoU row primitive (calculate_iou_batch_simple, train_yolo11_cuda.py:402-437)
    g = torch.Generator().manual_seed(5)
    b2 = torch.rand(4096, 4, generator=g) * 640
    b2 = torch.cat((b2[:, :2].minimum(b2[:, 2:]), b2[:, :2].maximum(b2[:, 2:])), 1)
    b1 = b2[17:18].clone()
    arrs["iou_b1"], arrs["iou_b2"] = b1, b2
    arrs["iou_out"] = ref_train.calculate_iou_batch_simple(b1, b2)
    save("nms.npz", **arrs)


def _pack_preds(preds):
    counts = np.asarray([len(p["scores"]) for p in preds], dtype=np.int64)
    boxes = torch.cat([p["boxes"].reshape(-1, 4) for p in preds]) if len(preds) else torch.zeros(0, 4)
    scores = torch.cat([p["scores"].reshape(-1) for p in preds])
    labels = torch.cat([p["labels"].reshape(-1) for p in preds])
    return counts, boxes, scores, labels


def gen_decode():
    arrs = {}
    am = synth.synth_eval_preds(2, 8400, seed=21)              # anchor-major (B, A, 9)
    out = ref_train.decode_predictions_for_metrics(am, 640, 0.25, 0.45, torch.device("cpu"))
    arrs["am_in"] = am
    arrs["am_counts"], arrs["am_boxes"], arrs["am_scores"], arrs["am_labels"] = _pack_preds(out)
    # literal call on the eval tensor layout (B, 4+nc, A)
    lit = am.transpose(1, 2).contiguous()
    out = ref_train.decode_predictions_for_metrics(lit, 640, 0.25, 0.45, torch.device("cpu"))
    arrs["lit_in"] = lit
    arrs["lit_counts"], arrs["lit_boxes"], arrs["lit_scores"], arrs["lit_labels"] = _pack_preds(out)
    save("decode.npz", **arrs)


# --------------------------------------------------------------------------- metrics
def gen_metrics():
    g = torch.Generator().manual_seed(31)
    preds, targets = [], []
    score_pool = torch.randperm(100000, generator=g).float() / 100000.0
    used = 0
    for i in range(12):
        nt = int(torch.randint(0, 9, (1,), generator=g))
        c = torch.rand(nt, 2, generator=g)
        wh = 0.05 + 0.2 * torch.rand(nt, 2, generator=g)
        tb = torch.cat((c - wh / 2, c + wh / 2), 1).clamp(0, 1)
        targets.append({"boxes": tb, "labels": torch.randint(0, 5, (nt,), generator=g)})
        npd = int(torch.randint(0, 14, (1,), generator=g))
        src = torch.randint(0, max(nt, 1), (npd,), generator=g)
        base = tb[src] if nt else torch.rand(npd, 4, generator=g)
        pb = (base + 0.03 * torch.randn(npd, 4, generator=g)).clamp(0, 1)
        ps = score_pool[used:used + npd].clone()
        used += npd
        preds.append({"boxes": pb, "scores": ps, "labels": torch.randint(0, 5, (npd,), generator=g)})
    res = evaluate_detections(copy.deepcopy(preds), copy.deepcopy(targets), 0.25, 0.5)
    pc, pbx, psc, plb = _pack_preds(preds)
    tc = np.asarray([len(t["boxes"]) for t in targets])
    save("metrics.npz", pred_counts=pc, pred_boxes=pbx, pred_scores=psc, pred_labels=plb,
         tgt_counts=tc, tgt_boxes=torch.cat([t["boxes"] for t in targets]),
         tgt_labels=torch.cat([t["labels"] for t in targets]),
         out=np.asarray([res["precision"], res["recall"], res["mAP50"], res["mAP50-95"]], np.float64))


# --------------------------------------------------------------------------- model fwd/loss/bwd
def gen_model(scale="n", imgsz=320, bs=2, name="model_n320.npz", full_grads=()):
    torch.manual_seed(0)
    m = build(scale)
    m.train()
    batch = synth.synth_batch(bs, imgsz, seed=7)
    crit = v8DetectionLoss(m, tal_topk=10)
    preds = m(batch["img"])
    heads = [p.detach().clone() for p in preds]
    loss, items = crit(preds, batch)
    loss.backward()
    arrs = dict(img=batch["img"], batch_idx=batch["batch_idx"], cls=batch["cls"], bboxes=batch["bboxes"],
                loss=loss.detach().reshape(1), items=items)
    for i, h in enumerate(heads):
        arrs[f"head{i}"] = h
    names, norms = [], []
    for k, p in m.named_parameters():
        names.append(k)
        norms.append(float(p.grad.norm()) if p.grad is not None else -1.0)
    arrs["grad_norm"] = np.asarray(norms, np.float64)
    arrs["grad_names"] = np.asarray(names)
    for k, p in m.named_parameters():
        if k in full_grads:
            arrs["grad:" + k] = p.grad
    sd = m.state_dict()
    for k in ("model.0.bn.running_mean", "model.0.bn.running_var", "model.10.m.0.attn.qkv.bn.running_var",
              "model.22.cv2.bn.running_mean", "model.23.cv3.2.1.bn.running_var"):
        arrs["state:" + k] = sd[k]
    # eval-mode decode output (Detect.inference, yolo11_modules.py:248-266), after the train step's BN update
    m.eval()
    with torch.no_grad():
        y, _ = m(batch["img"])
        vloss, vitems = crit(m(batch["img"]), batch)
    arrs["eval_y"] = y
    arrs["eval_loss"] = vloss.reshape(1)
    arrs["eval_items"] = vitems
    save(name, **arrs)


def gen_s_small():
    """s-scale graph pinned at a small resolution (channel widths, c3k, attention heads=4)."""
    m = build("s")
    m.train()
    batch = synth.synth_batch(1, 128, seed=8)
    preds = m(batch["img"])
    crit = v8DetectionLoss(m, tal_topk=10)
    loss, items = crit(preds, batch)
    loss.backward()
    arrs = dict(img=batch["img"], batch_idx=batch["batch_idx"], cls=batch["cls"], bboxes=batch["bboxes"],
                loss=loss.detach().reshape(1), items=items)
    for i, h in enumerate(preds):
        arrs[f"head{i}"] = h
    arrs["grad_norm"] = np.asarray([float(p.grad.norm()) if p.grad is not None else -1.0 for p in m.parameters()], np.float64)
    arrs["grad:model.10.m.0.attn.qkv.conv.weight"] = m.model[10].m[0].attn.qkv.conv.weight.grad
    arrs["grad:model.0.conv.weight"] = m.model[0].conv.weight.grad
    save("model_s128.npz", **arrs)


def gen_m_small():
    """m-scale graph (1024-channel layers, C2PSA heads=8) pinned at 256x256 bs1."""
    m = build("m")
    m.train()
    batch = synth.synth_batch(1, 256, seed=9)
    preds = m(batch["img"])
    crit = v8DetectionLoss(m, tal_topk=10)
    loss, items = crit(preds, batch)
    loss.backward()
    arrs = dict(img=batch["img"], batch_idx=batch["batch_idx"], cls=batch["cls"], bboxes=batch["bboxes"],
                loss=loss.detach().reshape(1), items=items)
    for i, h in enumerate(preds):
        arrs[f"head{i}"] = h
    arrs["grad_names"] = np.asarray([k for k, _ in m.named_parameters()])
    arrs["grad_norm"] = np.asarray([float(p.grad.norm()) if p.grad is not None else -1.0 for p in m.parameters()],
                                   np.float64)
    for k in ("model.0.conv.weight", "model.10.m.0.attn.qkv.conv.weight", "model.23.cv2.2.2.weight"):
        arrs["grad:" + k] = dict(m.named_parameters())[k].grad
    save("model_m256.npz", **arrs)


def gen_detect():
    """Detect called on its own (yolo11_modules.py:195-266): train-mode maps + backward, then the
    eval-mode (y, maps) after the BN running-stat update; and Concat (:277-285)."""
    torch.manual_seed(3)
    det = ref_mods.Detect(5, (32, 64, 128))
    det.stride = torch.tensor([8.0, 16.0, 32.0])
    for k, v in det.state_dict().items():
        if k.endswith(".weight") and v.dim() == 4:
            v.copy_(torch.randn(v.shape) * (2.0 / (v.shape[0] * v.shape[2] * v.shape[3])) ** 0.5)
    det.bias_init()
    det.apply(lambda m: setattr(m, "eps", 1e-3) if isinstance(m, torch.nn.BatchNorm2d) else None)
    det.apply(lambda m: setattr(m, "momentum", 0.03) if isinstance(m, torch.nn.BatchNorm2d) else None)
    arrs = {f"p:{k}": v.clone() for k, v in det.state_dict().items()}
    g = torch.Generator().manual_seed(61)
    shapes = [(2, 32, 16, 16), (2, 64, 8, 8), (2, 128, 4, 4)]
    xs = [torch.randn(s, generator=g).requires_grad_(True) for s in shapes]
    det.train()
    ys = det([x for x in xs])
    dys = [torch.randn(y.shape, generator=g) for y in ys]
    torch.autograd.backward(ys, dys)
    for i in range(3):
        arrs[f"x{i}"], arrs[f"y{i}"], arrs[f"dy{i}"], arrs[f"dx{i}"] = xs[i], ys[i], dys[i], xs[i].grad
    for k, p in det.named_parameters():
        if p.grad is not None:
            arrs[f"g:{k}"] = p.grad
    for k, v in det.state_dict().items():
        if "running" in k:
            arrs[f"s:{k}"] = v.clone()
    det.eval()
    with torch.no_grad():
        y, maps = det([x.detach() for x in xs])
    arrs["eval_y"] = y
    for i in range(3):
        arrs[f"eval_map{i}"] = maps[i]
    # Concat along dim 1 and dim 2
    cat = ref_mods.Concat(1)
    a, b = torch.randn(2, 3, 4, 5, generator=g), torch.randn(2, 6, 4, 5, generator=g)
    arrs.update(cat_a=a, cat_b=b, cat_out1=cat([a, b]), cat_out2=ref_mods.Concat(2)([a, a[:, :, :2]]))
    save("detect.npz", **arrs)


def _fingerprint(t: torch.Tensor, n: int = 16384) -> np.ndarray:
    """A fixed strided subsample of a large tensor (element-wise comparison on a subset)."""
    flat = t.detach().reshape(-1)
    step = max(1, flat.numel() // n)
    return flat[::step][:n].numpy().copy()


def gen_attn_big():
    """C2PSA at the attention shapes of the s@640 (heads=4, N=400) and m@1280 (heads=8, N=1600)
    configs.  Weights are key-seeded (oracle/weights.py), inputs and output gradients drawn from
    seeded CPU generators, so the fixture holds only outputs: per-tensor fingerprints (strided
    subsamples), norms and parameter-gradient norms."""
    arrs = {}
    cases = {"h4n400": (512, (2, 512, 20, 20), 51), "h8n1600": (1024, (1, 1024, 40, 40), 52)}
    for name, (c, shape, seed) in cases.items():
        mod = ref_mods.C2PSA(c, c, 1)
        apply_seeded_weights(mod.state_dict())
        mod.apply(lambda m: setattr(m, "eps", 1e-3) if isinstance(m, torch.nn.BatchNorm2d) else None)
        mod.apply(lambda m: setattr(m, "momentum", 0.03) if isinstance(m, torch.nn.BatchNorm2d) else None)
        mod.train()
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(shape, generator=g).requires_grad_(True)
        dy = torch.randn(shape, generator=g)
        y = mod(x)
        y.backward(dy)
        arrs[f"{name}/y_fp"] = _fingerprint(y)
        arrs[f"{name}/dx_fp"] = _fingerprint(x.grad)
        arrs[f"{name}/y_norm"] = np.float64(y.detach().double().norm())
        arrs[f"{name}/dx_norm"] = np.float64(x.grad.double().norm())
        arrs[f"{name}/grad_names"] = np.asarray([k for k, _ in mod.named_parameters()])
        arrs[f"{name}/grad_norm"] = np.asarray([float(p.grad.norm()) for p in mod.parameters()], np.float64)
        arrs[f"{name}/qkv_grad_fp"] = _fingerprint(mod.m[0].attn.qkv.conv.weight.grad)
    save("attn_big.npz", **arrs)


# --------------------------------------------------------------------------- per-block
def _block_case(mod, x, seed):
    mod.train()
    x = x.clone().requires_grad_(True)
    y = mod(x)
    g = torch.Generator().manual_seed(seed)
    if isinstance(y, list):
        dys = [torch.randn(t.shape, generator=g) for t in y]
        torch.autograd.backward(y, dys)
        return x, y, dys
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    return x, [y], [dy]


def gen_blocks():
    arrs = {}
    torch.manual_seed(1)
    cases = {
        "conv3s1": (lambda: ref_mods.Conv(32, 64, 3, 1), (2, 32, 12, 12)),
        "conv3s2": (lambda: ref_mods.Conv(32, 64, 3, 2), (2, 32, 13, 11)),
        "conv1": (lambda: ref_mods.Conv(64, 32, 1, 1), (2, 64, 9, 7)),
        "conv0": (lambda: ref_mods.Conv(1, 32, 3, 2), (2, 1, 16, 16)),
        "c3k2": (lambda: ref_mods.C3k2(64, 64, 1, False, 0.25), (2, 64, 10, 10)),
        "c3k2k": (lambda: ref_mods.C3k2(64, 128, 1, True), (2, 64, 8, 8)),
        "sppf": (lambda: ref_mods.SPPF(128, 128, 5), (2, 128, 8, 8)),
        "c2psa": (lambda: ref_mods.C2PSA(256, 256, 1), (2, 256, 5, 4)),
    }
    for name, (ctor, shape) in cases.items():
        mod = ctor()
        for k, v in mod.state_dict().items():
            if k.endswith(".weight") and v.dim() == 4:
                v.copy_(torch.randn(v.shape) * (2.0 / (v.shape[0] * v.shape[2] * v.shape[3])) ** 0.5)
            elif k.endswith("bn.weight"):
                v.copy_(1.0 + 0.1 * torch.randn(v.shape))
            elif k.endswith("bn.bias"):
                v.copy_(0.1 * torch.randn(v.shape))
        for k, v in mod.state_dict().items():
            arrs[f"{name}/p:{k}"] = v.clone()
        mod.apply(lambda m: setattr(m, "eps", 1e-3) if isinstance(m, torch.nn.BatchNorm2d) else None)
        mod.apply(lambda m: setattr(m, "momentum", 0.03) if isinstance(m, torch.nn.BatchNorm2d) else None)
        x = torch.randn(shape)
        x_, ys, dys = _block_case(mod, x, seed=3)
        arrs[f"{name}/x"] = x
        arrs[f"{name}/y"] = ys[0]
        arrs[f"{name}/dy"] = dys[0]
        arrs[f"{name}/dx"] = x_.grad
        for k, p in mod.named_parameters():
            arrs[f"{name}/g:{k}"] = p.grad
        for k, v in mod.state_dict().items():
            if "running" in k:
                arrs[f"{name}/s:{k}"] = v.clone()
    save("blocks.npz", **arrs)


# --------------------------------------------------------------------------- assigner / loss
class _StubModel(torch.nn.Module):
    def __init__(self, stride):
        super().__init__()
        self.det = ref_mods.Detect(5, (64, 128, 256))
        self.det.stride = torch.tensor(stride, dtype=torch.float32)


def gen_assigner():
    """Crafted targets at 320 (A=2100) that exercise loop 1, loop 2, empty images and M=max."""
    arrs = {}
    stub = _StubModel([8.0, 16.0, 32.0])
    crit = v8DetectionLoss(stub, tal_topk=10)
    g = torch.Generator().manual_seed(41)
    B, S = 3, 320
    shapes = [(B, 69, S // 8, S // 8), (B, 69, S // 16, S // 16), (B, 69, S // 32, S // 32)]
    feats = [torch.randn(s, generator=g) * 2.0 for s in shapes]
    bidx, cls, boxes = [], [], []
    # image 0: ordinary boxes + one tiny box between anchor centres (loop 1: no in-box anchor)
    b0 = [[0.10, 0.10, 0.40, 0.35], [0.50, 0.55, 0.90, 0.95], [0.6, 0.1, 0.8, 0.3],
          [0.2030, 0.2030, 0.2045, 0.2045], [0.05, 0.6, 0.3, 0.9]]
    # image 1: nested / shadowed boxes (loop 2) + many overlaps
    b1 = [[0.2, 0.2, 0.8, 0.8], [0.21, 0.21, 0.79, 0.79], [0.3, 0.3, 0.5, 0.5], [0.31, 0.31, 0.49, 0.49],
          [0.0, 0.0, 1.0, 1.0], [0.7, 0.7, 0.72, 0.72], [0.45, 0.1, 0.55, 0.2]]
    # image 2: no targets
    for i, bl in enumerate((b0, b1)):
        for j, b in enumerate(bl):
            bidx.append(i)
            cls.append([(i * 3 + j) % 5])
            boxes.append(b)
    batch = {"img": torch.zeros(B, 1, S, S), "batch_idx": torch.tensor(bidx), "cls": torch.tensor(cls),
             "bboxes": torch.tensor(boxes, dtype=torch.float32)}
    feats_in = [f.clone().requires_grad_(True) for f in feats]
    # capture the assigner's outputs
    captured = {}
    orig = crit.assigner.forward

    def spy(*a, **k):
        captured["as_in"] = [t.detach().clone() for t in a]
        r = orig(*a, **k)
        captured["r"] = tuple(t.clone() for t in r)       # the loss divides target_bboxes in place (:479)
        return r

    crit.assigner.forward = spy
    orig_bl = crit.bbox_loss.forward

    def spy_bl(*a, **k):
        captured["bl_in"] = [t.detach().clone() if isinstance(t, torch.Tensor) else t for t in a]
        r = orig_bl(*a, **k)
        captured["bl_out"] = [t.detach().clone() for t in r]
        return r

    crit.bbox_loss.forward = spy_bl
    loss, items = crit(feats_in, batch)
    loss.backward()
    tl, tb, ts, fg, tgi = captured["r"]
    # the assigner's own inputs (TaskAlignedAssigner.forward, yolo_v8_loss.py:78-180)
    for nm, t in zip(("pd_scores", "pd_bboxes", "anc_points", "gt_labels", "gt_bboxes", "mask_gt"), captured["as_in"]):
        arrs["as_" + nm] = t
    # BboxLoss.forward (:280-310) inputs / outputs, and its gradient w.r.t. pred_dist and pred_bboxes for
    # the seed 1.3 * d loss_iou + 0.7 * d loss_dfl
    pd, pb, ap, tbb, tsc, tss, fgm = captured["bl_in"]
    arrs.update(bl_pred_dist=pd, bl_pred_bboxes=pb, bl_anchor_points=ap, bl_target_bboxes=tbb,
                bl_target_scores=tsc, bl_tss=np.float32(float(tss)), bl_fg_mask=fgm,
                bl_loss_iou=captured["bl_out"][0], bl_loss_dfl=captured["bl_out"][1])
    pdl, pbl = pd.clone().requires_grad_(True), pb.clone().requires_grad_(True)
    li, ld = ref_loss_mod.BboxLoss(16)(pdl, pbl, ap, tbb.clone(), tsc, tss, fgm)
    (1.3 * li + 0.7 * ld).backward()
    arrs.update(bl_dpred_dist=pdl.grad, bl_dpred_bboxes=pbl.grad)
    for i, f in enumerate(feats):
        arrs[f"feat{i}"] = f
        arrs[f"dfeat{i}"] = feats_in[i].grad
    arrs.update(batch_idx=batch["batch_idx"], cls=batch["cls"], bboxes=batch["bboxes"],
                fg=fg, tgi=tgi, target_scores=ts, target_bboxes=tb, target_labels=tl,
                loss=loss.detach().reshape(1), items=items)
    # empty batch (M = 0)
    empty = {"img": batch["img"], "batch_idx": torch.zeros(0, dtype=torch.long),
             "cls": torch.zeros(0, 1, dtype=torch.long), "bboxes": torch.zeros(0, 4)}
    feats_e = [f.clone().requires_grad_(True) for f in feats]
    le, ie = crit(feats_e, empty)
    le.backward()
    arrs["empty_loss"], arrs["empty_items"] = le.detach().reshape(1), ie
    for i in range(3):
        arrs[f"empty_dfeat{i}"] = feats_e[i].grad
    save("assigner.npz", **arrs)


def gen_modules():
    """Module classes called on their own (models/__init__.py and losses/__init__.py exports):
    Attention.forward (yolo11_modules.py:124-136) at the PSA head shape (heads=4) and at the class
    default heads=8, train-mode forward + backward; DFL.forward (:189-192) with the arange weights
    it is built with and with Kaiming weights (as _initialize_weights leaves them, Q5), forward +
    input gradient; TaskAlignedAssigner with its class defaults (alpha=1.0, beta=6.0,
    yolo_v8_loss.py:67) on the assigner fixture's inputs."""
    arrs = {}
    for name, (dim, heads, shape, seed) in {"attn_h4": (256, 4, (2, 256, 20, 20), 71),
                                            "attn_h8": (512, 8, (1, 512, 10, 12), 72)}.items():
        mod = ref_mods.Attention(dim, num_heads=heads, attn_ratio=0.5)
        apply_seeded_weights(mod.state_dict())
        mod.apply(lambda m: setattr(m, "eps", 1e-3) if isinstance(m, torch.nn.BatchNorm2d) else None)
        mod.apply(lambda m: setattr(m, "momentum", 0.03) if isinstance(m, torch.nn.BatchNorm2d) else None)
        # weights are key-seeded (oracle/weights.py) and x / dy come from seeded CPU generators
        # (x: Generator(seed), dy: Generator(seed + 100)), so the test re-creates them; stored: outputs
        x, ys, dys = _block_case(mod, torch.randn(shape, generator=torch.Generator().manual_seed(seed)), seed + 100)
        arrs[f"{name}/y"], arrs[f"{name}/dx"] = ys[0], x.grad
        for k, p in mod.named_parameters():
            if p.grad.numel() > 65536:      # large weight gradients: strided fingerprint + norm
                arrs[f"{name}/gfp:{k}"] = _fingerprint(p.grad)
                arrs[f"{name}/gn:{k}"] = np.float64(p.grad.double().norm())
            else:
                arrs[f"{name}/g:{k}"] = p.grad
        for k, v in mod.state_dict().items():
            if "running" in k:
                arrs[f"{name}/s:{k}"] = v.clone()
    g = torch.Generator().manual_seed(73)
    for name, kaiming in (("dfl_arange", False), ("dfl_kaiming", True)):
        mod = ref_mods.DFL(16)
        if kaiming:
            torch.nn.init.kaiming_normal_(mod.conv.weight, generator=g, mode="fan_out", nonlinearity="relu")
        x = (torch.randn(2, 64, 300, generator=g) * 3.0).requires_grad_(True)
        y = mod(x)
        dy = torch.randn(y.shape, generator=g)
        y.backward(dy)
        arrs.update({f"{name}/w": mod.conv.weight.detach().reshape(-1), f"{name}/x": x, f"{name}/y": y,
                     f"{name}/dy": dy, f"{name}/dx": x.grad})
    a = np.load(HERE / "assigner.npz")
    ins = [torch.from_numpy(a["as_" + k]) for k in ("pd_scores", "pd_bboxes", "anc_points", "gt_labels", "gt_bboxes",
                                                   "mask_gt")]
    tal = ref_loss_mod.TaskAlignedAssigner(num_classes=5)
    for nm, t in zip(("target_labels", "target_bboxes", "target_scores", "fg_mask", "target_gt_idx"), tal(*ins)):
        arrs[f"tal_default/{nm}"] = t
    arrs["tal_default/params"] = np.asarray([tal.alpha, tal.beta, tal.eps], np.float64)
    save("modules.npz", **arrs)


# --------------------------------------------------------------------------- loss curve
def gen_curve(steps=20):
    torch.manual_seed(0)
    m = build("n")
    crit = v8DetectionLoss(m, tal_topk=10)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=5e-4)
    rows, sums = [], []
    m.train()
    for step in range(steps):
        batch = synth.synth_batch(4, 320, seed=100 + step)
        sums.append([float(batch["img"].double().sum()), float(batch["bboxes"].double().sum()), len(batch["cls"])])
        opt.zero_grad(set_to_none=True)
        preds = m(batch["img"])
        loss, items = crit(preds, batch)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(m.parameters(), max_norm=10.0)
        opt.step()
        rows.append([float(loss), *[float(v) for v in items], float(gn)])
        print(f"  step {step}: loss {rows[-1][0]:.4f} gn {rows[-1][-1]:.2f}")
    save("curve.npz", rows=np.asarray(rows), batch_sums=np.asarray(sums))


if __name__ == "__main__":
    which = sys.argv[1:] or ["structure", "nms", "decode", "metrics", "model", "s_small", "m_small", "attn_big",
                             "detect", "blocks", "assigner", "modules", "curve"]
    if "structure" in which:
        gen_structure()
    if "nms" in which:
        gen_nms()
    if "decode" in which:
        gen_decode()
    if "metrics" in which:
        gen_metrics()
    if "model" in which:
        gen_model(full_grads=("model.0.conv.weight", "model.23.cv2.0.2.weight", "model.23.cv3.0.2.bias",
                              "model.10.m.0.attn.qkv.conv.weight", "model.2.m.0.cv1.bn.weight"))
    if "s_small" in which:
        gen_s_small()
    if "m_small" in which:
        gen_m_small()
    if "attn_big" in which:
        gen_attn_big()
    if "detect" in which:
        gen_detect()
    if "blocks" in which:
        gen_blocks()
    if "assigner" in which:
        gen_assigner()
    if "modules" in which:
        gen_modules()
    if "curve" in which:
        gen_curve()
