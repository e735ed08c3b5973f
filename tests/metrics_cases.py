"""Inputs for the detection-metrics parity tests (oracle/metrics.py vs utils/metrics.py).

golden_case(): the committed reference run (tests/golden/metrics.npz, made by the reference's
own evaluate_detections in tests/golden/gen_golden.py:gen_metrics).
random_case(): seeded images with GT boxes and jittered / duplicated / spurious predictions,
scores quantised so equal scores occur within and across images (the TP-before-FP rule of
calculate_ap's stable sort), images without GT, without predictions, and below-conf scores."""
import numpy as np
import torch


def split(counts, *arrays):
    out, off = [], 0
    for c in counts:
        out.append([a[off:off + c] for a in arrays])
        off += c
    return out


def golden_case(d):
    preds = [{"boxes": torch.from_numpy(b), "scores": torch.from_numpy(s), "labels": torch.from_numpy(l)}
             for b, s, l in split(d["pred_counts"], d["pred_boxes"], d["pred_scores"], d["pred_labels"])]
    tgts = [{"boxes": torch.from_numpy(b), "labels": torch.from_numpy(l)}
            for b, l in split(d["tgt_counts"], d["tgt_boxes"], d["tgt_labels"])]
    return preds, tgts


def random_case(seed, n_img=60, max_gt=25, max_pred=50, quant=32):
    rng = np.random.default_rng(seed)
    preds, tgts = [], []
    for i in range(n_img):
        nt = int(rng.integers(0, max_gt + 1)) if i % 7 else 0
        c = rng.random((nt, 2))
        wh = 0.02 + 0.2 * rng.random((nt, 2))
        tb = np.clip(np.concatenate([c - wh / 2, c + wh / 2], 1), 0, 1).astype(np.float32)
        npd = int(rng.integers(0, max_pred + 1)) if i % 11 else 0
        if nt:
            src = rng.integers(0, nt, npd)
            pb = tb[src] + rng.normal(0, 0.02, (npd, 4))
            spurious = rng.random(npd) < 0.2
            pb[spurious] = rng.random((int(spurious.sum()), 4))
        else:
            pb = rng.random((npd, 4))
        pb = np.stack([np.minimum(pb[:, 0], pb[:, 2]), np.minimum(pb[:, 1], pb[:, 3]),
                       np.maximum(pb[:, 0], pb[:, 2]), np.maximum(pb[:, 1], pb[:, 3])], 1).astype(np.float32)
        ps = (np.floor(rng.random(npd) * quant) / quant).astype(np.float32)   # ties; some < conf
        preds.append({"boxes": torch.from_numpy(pb), "scores": torch.from_numpy(ps),
                      "labels": torch.zeros(npd, dtype=torch.int64)})
        tgts.append({"boxes": torch.from_numpy(tb), "labels": torch.zeros(nt, dtype=torch.int64)})
    return preds, tgts
