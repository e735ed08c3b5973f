"""Train YOLOv11 on MI355X — drop-in for the reference entry point.

Same CLI flags, same functions and return conventions as the reference's
train_yolo11_cuda.py (/root/reference/yolo_scratch_cuda/train_yolo11_cuda.py):
train_one_epoch :31-98, validate :101-262, decode_predictions_for_metrics
:265-358, nms_simple :361-399, calculate_iou_batch_simple :402-437,
cosine_lr_schedule :440-451, main :454-661.

What differs underneath: the model forward/backward, the loss and the decode +
NMS postprocess run as hand-written HIP kernels for gfx950 (libyolomi.so);
per-step loss items are accumulated on the device and read back every
`LOG_EVERY` steps instead of four host syncs per step; `--synthetic N` trains
on N synthetic batches when no dataset is mounted; multi-GPU data parallelism
is enabled by launching with torchrun (one process per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import math
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).parent))

from models.yolo11_model import build_yolo11  # noqa: E402
from losses.yolo_v8_loss import v8DetectionLoss  # noqa: E402
from datasets import collate_fn_cuda, prepare_batch  # noqa: E402
from utils.metrics import evaluate_detections  # noqa: E402
from yolomi import post as _post  # noqa: E402

collate_fn = collate_fn_cuda
LOG_EVERY = 10


def _tqdm(it, **kw):
    try:
        from tqdm import tqdm
        return tqdm(it, **kw)
    except Exception:  # pragma: no cover
        return it


def train_one_epoch(model, dataloader, optimizer, criterion, device, epoch, epochs, dp=None):
    """One epoch (reference :31-98).  `dp` is an optional yolomi.dist.GradSync."""
    model.train()
    pbar = _tqdm(dataloader, desc=f"Epoch {epoch}/{epochs}")
    sums = torch.zeros(4, device=device)
    n = 0
    for batch_idx, batch in enumerate(pbar):
        batch = prepare_batch(batch, device)        # H2D (+ GPU resize of raw images)
        optimizer.zero_grad(set_to_none=True)
        preds = model(batch["img"])
        loss, loss_items = criterion(preds, batch)
        loss.backward()
        if dp is not None:
            dp.sync()
        if not getattr(optimizer, "fuses_clip", False):    # FusedAdamW clips on the device itself
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=10.0)
        optimizer.step()
        sums[0] += loss.detach()
        sums[1:] += loss_items.detach()
        n += 1
        if hasattr(pbar, "set_postfix") and (batch_idx + 1) % LOG_EVERY == 0:
            s = (sums / n).tolist()
            pbar.set_postfix({"loss": f"{s[0]:.4f}", "box": f"{s[1]:.4f}", "cls": f"{s[2]:.4f}", "dfl": f"{s[3]:.4f}"})
    s = (sums / max(len(dataloader), 1)).tolist()
    return {"loss": s[0], "box_loss": s[1], "cls_loss": s[2], "dfl_loss": s[3]}


@torch.no_grad()
def validate(model, dataloader, criterion, device, conf_threshold=0.25, iou_threshold=0.45, max_batches=None,
             dp=None):
    """Validation + metrics (reference :101-262).  Under data parallelism (`dp`, a GradSync) each
    rank evaluates its ValShard of the val set (decode + NMS on its own GPU), the per-image
    detections are gathered to rank 0 in the global image order and evaluate_detections runs there
    (SURVEY §8(e)); the loss sums are all-reduced and the metrics broadcast, so every rank returns
    the same dict."""
    model.eval()
    sums = torch.zeros(4, device=device)
    all_predictions, all_targets = [], []
    batches = 0
    for batch in _tqdm(dataloader, desc="Validating"):
        batch = prepare_batch(batch, device)
        preds = model(batch["img"])
        loss, loss_items = criterion(preds, batch)
        sums[0] += loss
        sums[1:] += loss_items
        if isinstance(preds, tuple) and len(preds) == 2:
            predictions = decode_predictions_for_metrics(preds[0], batch["img"].shape[-1], conf_threshold,
                                                         iou_threshold, device)
        else:
            decoded = model(batch["img"])
            predictions = decode_predictions_for_metrics(decoded[0], batch["img"].shape[-1], conf_threshold,
                                                         iou_threshold, device)
        all_predictions.extend(predictions)
        bidx, bboxes, cls = batch["batch_idx"], batch["bboxes"], batch["cls"]
        for i in range(batch["img"].shape[0]):
            m = bidx == i
            all_targets.append({"boxes": bboxes[m], "labels": cls[m].reshape(-1)})
        batches += 1
        if max_batches is not None and batches >= max_batches:
            break
    nb = torch.tensor([float(batches)], device=device)
    world = dp.ctx.world if dp is not None else 1
    if world > 1:
        import torch.distributed as tdist
        from yolomi.dist import gather_detections
        tdist.all_reduce(sums)
        tdist.all_reduce(nb)
        all_predictions, all_targets = gather_detections(all_predictions, all_targets, dp.ctx, device)
    keys = ("precision", "recall", "mAP50", "mAP50-95")
    if all_predictions is not None:
        # predictions and targets stay in HBM: the metrics run on the GPU (utils/metrics.py)
        metrics = evaluate_detections(all_predictions, all_targets, conf_threshold=conf_threshold, iou_threshold=0.5)
    if world > 1:
        mt = torch.tensor([float(metrics[k]) for k in keys] if all_predictions is not None else [0.0] * 4,
                          dtype=torch.float64, device=device)
        tdist.broadcast(mt, 0)
        metrics = dict(zip(keys, mt.tolist()))
    nbatch = float(nb) if (max_batches or world > 1) else len(dataloader)
    s = (sums / max(nbatch, 1)).tolist()
    return {"loss": s[0], "box_loss": s[1], "cls_loss": s[2], "dfl_loss": s[3], **metrics}


def decode_predictions_for_metrics(preds, img_size, conf_threshold, iou_threshold, device):
    """Per-image boxes/scores/labels (normalised xyxy) from decoded predictions.

    Reads `preds` as (batch, rows, 4+C) exactly like the reference (:289-301),
    including when it is handed the (B, 4+nc, A) eval tensor.
    One batched GPU launch pair; one host sync for the per-image counts.
    """
    pred = preds[0] if isinstance(preds, tuple) and len(preds) == 2 else preds
    return _post.decode_nms(pred, img_size, conf_threshold, iou_threshold)


def nms_simple(boxes, scores, iou_threshold):
    """Greedy class-agnostic NMS; returns the list of kept indices (reference :361-399)."""
    if len(boxes) == 0:
        return []
    return _post.nms(boxes, scores, iou_threshold).cpu().tolist()


def calculate_iou_batch_simple(boxes1, boxes2):
    """IoU of boxes1 (1,4) against boxes2 (M,4) (reference :402-437)."""
    if boxes1.dim() == 1:
        boxes1 = boxes1.unsqueeze(0)
    rows = [_post.iou_row(b, boxes2) for b in boxes1]
    iou = torch.stack(rows) if rows else boxes2.new_zeros(0, boxes2.shape[0])
    return iou.squeeze() if iou.dim() > 1 and iou.shape[0] == 1 else iou


def cosine_lr_schedule(optimizer, epoch, epochs, lr_min=1e-6, lr_max=1e-3, warmup_epochs=3):
    """Per-epoch cosine schedule with linear warm-up (reference :440-451)."""
    if epoch < warmup_epochs:
        lr = lr_min + (lr_max - lr_min) * (epoch / warmup_epochs)
    else:
        progress = (epoch - warmup_epochs) / (epochs - warmup_epochs)
        lr = lr_min + (lr_max - lr_min) * 0.5 * (1 + math.cos(math.pi * progress))
    for g in optimizer.param_groups:
        g["lr"] = lr
    return lr


def make_checkpoint(epoch, model, optimizer, train_metrics, val_metrics, best_loss, best_mAP50):
    """The reference's checkpoint dict (train_yolo11_cuda.py:628-636), key for key: last.pt / best.pt
    written by either implementation resume in the other (tests/test_models_cpu.py)."""
    return {"epoch": epoch, "model_state_dict": model.state_dict(), "optimizer_state_dict": optimizer.state_dict(),
            "train_metrics": train_metrics, "val_metrics": val_metrics, "best_loss": best_loss,
            "best_mAP50": best_mAP50}


def _np_safe_globals():
    """numpy scalar reconstructors a reference-written checkpoint needs: its evaluate_detections
    returns np.float64 mAP values (utils/metrics.py:264-274) that end up in val_metrics and
    best_mAP50.  These rebuild plain numbers; nothing else is allowed through the restricted loader."""
    import numpy as np
    out = [np.dtype, type(np.dtype(np.float64)), type(np.dtype(np.float32)), type(np.dtype(np.int64))]
    for mod in ("numpy._core.multiarray", "numpy.core.multiarray"):
        try:
            m = __import__(mod, fromlist=["scalar"])
            out.append(m.scalar)
            break
        except (ImportError, AttributeError):
            continue
    return out



def _load_np_safe(path, device):
    with torch.serialization.safe_globals(_np_safe_globals()):
        return torch.load(path, map_location=device, weights_only=True)


def resume_checkpoint(path, model, optimizer, device):
    """Resume as the reference does (:576-586) -> (start_epoch, best_loss, best_mAP50).  Loaded with
    weights_only=True plus the numpy scalar types a reference-written checkpoint holds (its metrics
    are np.float64); the optimizer keeps this process's fused/foreach implementation choice across a
    reference-written state."""
    ckpt = _load_np_safe(path, device)
    model.load_state_dict(ckpt["model_state_dict"])
    impl = [{k: g.get(k) for k in ("fused", "foreach")} for g in optimizer.param_groups]
    optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    for g, kv in zip(optimizer.param_groups, impl):
        g.update(kv)
    return ckpt["epoch"] + 1, ckpt.get("best_loss", float("inf")), ckpt.get("best_mAP50", 0.0)


def make_loaders(dataset, val_split, batch, workers, imgsz, dp_ctx=None, collate=None):
    """The reference's split and loaders (:491-543): seed-42 permutation, Subset train / val,
    shuffled train loader, ordered val loader, drop_last=False.  Under data parallelism the train set
    is sharded by a DistributedSampler(shuffle=True, drop_last=True): every rank gets the same number
    of samples and so the same number of batches (a rank with one batch more would enter the gradient
    all-reduce alone and hang), reshuffled every epoch (set_epoch); the val set by ValShard (no
    padding: no image counted twice).  -> (train_loader, val_loader, train_sampler or None)."""
    import functools
    from torch.utils.data import DataLoader, DistributedSampler, Subset
    n = len(dataset)
    val_size = int(n * val_split)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(42)).tolist()
    tr, va = Subset(dataset, idx[: n - val_size]), Subset(dataset, idx[n - val_size:])
    nw = min(workers, 4)
    col = collate or functools.partial(collate_fn, img_size=imgsz)
    kw = dict(batch_size=batch, num_workers=nw, collate_fn=col, pin_memory=torch.cuda.is_available(),
              persistent_workers=nw > 0, prefetch_factor=2 if nw > 0 else None, drop_last=False)
    if dp_ctx is not None and dp_ctx.world > 1:
        from yolomi.dist import ValShard
        sampler = DistributedSampler(tr, num_replicas=dp_ctx.world, rank=dp_ctx.rank, shuffle=True, seed=0,
                                     drop_last=True)
        return (DataLoader(tr, sampler=sampler, **kw),
                DataLoader(va, sampler=ValShard(len(va), dp_ctx.rank, dp_ctx.world), **kw), sampler)
    return DataLoader(tr, shuffle=True, **kw), DataLoader(va, shuffle=False, **kw), None


class _SyntheticLoader:
    def __init__(self, n, batch, imgsz, seed):
        from datasets.synthetic import synth_batch
        self._mk = lambda i: synth_batch(batch, imgsz, seed + i)
        self.n = n

    def __len__(self):
        return self.n

    def __iter__(self):
        for i in range(self.n):
            yield self._mk(i)


def main():
    ap = argparse.ArgumentParser(description="Train YOLOv11 for Crater Detection (MI355X)")
    ap.add_argument("--data", type=str, default="/content/data/train")
    ap.add_argument("--cfg", type=str, default=str(Path(__file__).parent / "configs" / "yolo11n_crater.yaml"))
    ap.add_argument("--scale", type=str, default="s", choices=["n", "s", "m", "l", "x"])
    ap.add_argument("--epochs", type=int, default=150)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--device", type=str, default="cuda")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--lr", type=float, default=0.001)
    ap.add_argument("--weight-decay", type=float, default=0.0005)
    ap.add_argument("--val-split", type=float, default=0.2)
    ap.add_argument("--save-dir", type=str, default="/content/drive/MyDrive/YOLO11_crater_cuda")
    ap.add_argument("--resume", type=str, default="/content/drive/MyDrive/YOLO11_crater_cuda/last.pt")
    ap.add_argument("--max-val-batches", type=int, default=None)
    ap.add_argument("--val-conf", type=float, default=0.25)
    ap.add_argument("--synthetic", type=int, default=0, help="train on N synthetic batches (no dataset needed)")
    args = ap.parse_args()

    from yolomi import dist as ydist
    dp_ctx = ydist.init_from_env()
    if not torch.cuda.is_available():
        raise SystemExit("yolomi runs on MI355X GPUs only (no CPU fallback)")
    device = torch.device("cuda", dp_ctx.local_rank if dp_ctx else 0)
    torch.cuda.set_device(device)
    rank0 = dp_ctx is None or dp_ctx.rank == 0
    save_dir = Path(args.save_dir)
    if rank0:
        save_dir.mkdir(parents=True, exist_ok=True)

    if args.synthetic:
        seed = 1000 * (dp_ctx.rank if dp_ctx else 0)
        train_loader = _SyntheticLoader(args.synthetic, args.batch, args.imgsz, seed)
        val_loader = _SyntheticLoader(max(1, args.synthetic // 5), args.batch, args.imgsz, seed + 10 ** 6)
        train_sampler = None
    else:
        from datasets import CraterDatasetCUDA
        dataset = CraterDatasetCUDA(args.data, img_size=args.imgsz, cache_images=False, augment=True)
        train_loader, val_loader, train_sampler = make_loaders(dataset, args.val_split, args.batch, args.workers,
                                                               args.imgsz, dp_ctx)

    import yaml
    with open(args.cfg) as f:
        cfg_dict = yaml.safe_load(f)
    cfg_dict["scale"] = args.scale
    model = build_yolo11(cfg=cfg_dict, ch=1, nc=5).to(device)
    if rank0:
        n_params = sum(p.numel() for p in model.parameters())
        print(f"Total parameters: {n_params:,} ({n_params / 1e6:.2f}M)")
    criterion = v8DetectionLoss(model, tal_topk=10)
    # the reference's AdamW (:440-451) + clip_grad_norm_(10) (:58-62): on the GPU as yolomi's
    # FusedAdamW (a torch.optim.AdamW with the same state_dict; clipping fused into its step)
    if device.type == "cuda":
        from yolomi.optim import FusedAdamW
        optimizer = FusedAdamW(model.parameters(), lr=args.lr, weight_decay=args.weight_decay, max_grad_norm=10.0)
    else:
        optimizer = torch.optim.AdamW(model.parameters(), lr=args.lr, weight_decay=args.weight_decay)
    dp = ydist.GradSync(model, dp_ctx) if dp_ctx else None
    start_epoch, best_loss, best_mAP50 = 0, float("inf"), 0.0
    if args.resume and os.path.isfile(args.resume):
        start_epoch, best_loss, best_mAP50 = resume_checkpoint(args.resume, model, optimizer, device)
        if rank0:
            print(f"Resumed from epoch {start_epoch}, best_loss={best_loss:.4f}, best_mAP50={best_mAP50:.4f}")
    if dp:
        dp.broadcast_state()

    for epoch in range(start_epoch, args.epochs):
        lr = cosine_lr_schedule(optimizer, epoch, args.epochs, lr_min=args.lr * 0.01, lr_max=args.lr, warmup_epochs=3)
        criterion.epoch = epoch
        if train_sampler is not None:
            train_sampler.set_epoch(epoch)
        tm = train_one_epoch(model, train_loader, optimizer, criterion, device, epoch + 1, args.epochs, dp)
        if dp:
            dp.sync_buffers()          # rank 0's BN running statistics for validation and the checkpoint
        vm = validate(model, val_loader, criterion, device, conf_threshold=args.val_conf, iou_threshold=0.45,
                      max_batches=args.max_val_batches, dp=dp)
        if not rank0:
            continue
        print(f"\nEpoch {epoch + 1}/{args.epochs} | LR: {lr:.6f}")
        print(f"  Train - Loss: {tm['loss']:.4f}, Box: {tm['box_loss']:.4f}, Cls: {tm['cls_loss']:.4f}, "
              f"DFL: {tm['dfl_loss']:.4f}")
        print(f"  Val   - Loss: {vm['loss']:.4f}, Box: {vm['box_loss']:.4f}, Cls: {vm['cls_loss']:.4f}, "
              f"DFL: {vm['dfl_loss']:.4f}")
        print(f"  Metrics - P: {vm.get('precision', 0.0):.4f}, R: {vm.get('recall', 0.0):.4f}, "
              f"mAP50: {vm.get('mAP50', 0.0):.4f}, mAP50-95: {vm.get('mAP50-95', 0.0):.4f}")
        ckpt = make_checkpoint(epoch, model, optimizer, tm, vm, best_loss, best_mAP50)
        torch.save(ckpt, save_dir / "last.pt")
        if "mAP50" in vm:
            if vm["mAP50"] > best_mAP50:
                best_mAP50 = vm["mAP50"]
                ckpt["best_mAP50"] = best_mAP50
                torch.save(ckpt, save_dir / "best.pt")
        elif vm["loss"] < best_loss:
            best_loss = vm["loss"]
            ckpt["best_loss"] = best_loss
            torch.save(ckpt, save_dir / "best.pt")
    if dp_ctx:
        ydist.shutdown()


if __name__ == "__main__":
    main()
