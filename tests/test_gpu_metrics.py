"""GPU detection metrics (utils/metrics.py -> csrc/metrics.hip) against the oracle.

Integer work (which prediction is a TP at which IoU threshold, the TP / FP counts,
precision and recall) must be bit-exact; APs are fp64 sums whose order differs from
numpy's pairwise sum, so they are compared to 1e-12 relative.  The reference's own run
(tests/golden/metrics.npz) is matched the same way."""
import numpy as np
import pytest
import torch

from metrics_cases import golden_case, random_case

pytestmark = pytest.mark.gpu
AP_RTOL = 1e-12


def _both(preds, tgts, conf=0.25, iou=0.5):
    from oracle import metrics as omet
    from utils import metrics as um
    ref = omet.evaluate_detections(preds, tgts, conf, iou, per_threshold=True)
    pb = torch.cat([p["boxes"].reshape(-1, 4) for p in preds]) if preds else torch.zeros(0, 4)
    ps = torch.cat([p["scores"].reshape(-1) for p in preds]) if preds else torch.zeros(0)
    gb = torch.cat([t["boxes"].reshape(-1, 4) for t in tgts]) if tgts else torch.zeros(0, 4)
    got = um.evaluate_packed(pb.cuda(), ps.cuda(), [len(p["boxes"]) for p in preds], gb.cuda(),
                             [len(t["boxes"]) for t in tgts], conf, iou)
    return ref, got


def _check(ref, got):
    assert got["tp50"] == ref["tp50"] and got["fp50"] == ref["fp50"]
    assert got["precision"] == ref["precision"] and got["recall"] == ref["recall"]
    np.testing.assert_allclose(got["ap"], ref["ap"], rtol=AP_RTOL, atol=1e-15)
    assert got["mAP50"] == pytest.approx(ref["mAP50"], rel=AP_RTOL, abs=1e-15)
    assert got["mAP50-95"] == pytest.approx(ref["mAP50-95"], rel=AP_RTOL, abs=1e-15)


def test_reference_golden_run(golden):
    from utils import metrics as um
    d = golden("metrics.npz")
    preds, tgts = golden_case(d)
    r = um.evaluate_detections(preds, tgts, 0.25, 0.5)          # CPU dicts, as the reference is called
    got = [r["precision"], r["recall"], r["mAP50"], r["mAP50-95"]]
    assert got[:2] == list(d["out"][:2])
    np.testing.assert_allclose(got[2:], d["out"][2:], rtol=AP_RTOL)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_random_sets_match_oracle(seed):
    preds, tgts = random_case(seed)
    ref, got = _both(preds, tgts)
    assert ref["tp50"] > 0 and ref["fp50"] > 0
    _check(ref, got)


@pytest.mark.parametrize("iou,conf", [(0.3, 0.25), (0.75, 0.1), (0.5, 0.0), (0.5, 0.9)])
def test_other_thresholds(iou, conf):
    preds, tgts = random_case(11, n_img=40)
    ref, got = _both(preds, tgts, conf, iou)
    _check(ref, got)


def test_many_gt_per_image():
    """More GT boxes than the LDS stage holds (2048) -> the L2 path; 64-bit masks up to 4096."""
    preds, tgts = random_case(5, n_img=3, max_gt=3000, max_pred=400, quant=1024)
    ref, got = _both(preds, tgts)
    _check(ref, got)


def test_edge_cases():
    e4, e = torch.zeros(0, 4), torch.zeros(0)
    box = torch.tensor([[0.1, 0.1, 0.4, 0.4]])
    # no predictions anywhere / no GT anywhere / everything below conf / no images
    cases = [
        ([{"boxes": e4, "scores": e}] * 3, [{"boxes": box}] * 3),
        ([{"boxes": box, "scores": torch.tensor([0.9])}] * 2, [{"boxes": e4}] * 2),
        ([{"boxes": box, "scores": torch.tensor([0.1])}], [{"boxes": box}]),
        ([{"boxes": box, "scores": torch.tensor([0.9])}], [{"boxes": box}]),
    ]
    for preds, tgts in cases:
        ref, got = _both(preds, tgts)
        _check(ref, got)
    from utils import metrics as um
    r = um.evaluate_detections([], [], 0.25, 0.5) if torch.cuda.is_available() else None
    assert r == {"precision": 0.0, "recall": 0.0, "mAP50": 0.0, "mAP50-95": 0.0}


def test_perfect_predictions_full_size():
    """5000 images x up to 100 GT, every GT predicted exactly with distinct scores: every
    prediction is a TP at every threshold, AP_t = sum_j (1/n) * max_{k>=j} k/(k+1e-6)."""
    from utils import metrics as um
    rng = np.random.default_rng(7)
    counts = rng.integers(0, 101, 5000)
    n = int(counts.sum())
    c = rng.random((n, 2))
    wh = 0.01 + 0.1 * rng.random((n, 2))
    gb = torch.from_numpy(np.concatenate([c - wh / 2, c + wh / 2], 1).astype(np.float32))
    ps = torch.from_numpy((rng.permutation(n) + 1).astype(np.float32) / np.float32(n + 1))
    r = um.evaluate_packed(gb.cuda(), ps.cuda(), counts.tolist(), gb.cuda(), counts.tolist(), 0.0, 0.5)
    k = np.arange(1, n + 1, dtype=np.float64)
    prec = k / (k + 1e-6)
    env = np.maximum.accumulate(prec[::-1])[::-1]
    ap = float(np.sum((k / n - (k - 1) / n) * env))
    assert r["tp50"] == n and r["fp50"] == 0 and r["n_valid"] == n
    np.testing.assert_allclose(r["ap"], [ap] * 10, rtol=1e-11)


def test_calculate_ap_and_iou_batch():
    from oracle import metrics as omet
    from utils import metrics as um
    rng = np.random.default_rng(3)
    for n_tp, n_fp, n_gt in [(0, 0, 5), (3, 0, 0), (40, 60, 50), (3000, 2000, 4000)]:
        tp = (np.floor(rng.random(n_tp) * 16) / 16).astype(np.float32).tolist()
        fp = (np.floor(rng.random(n_fp) * 16) / 16).astype(np.float32).tolist()
        assert um.calculate_ap(tp, fp, n_gt) == pytest.approx(omet.calculate_ap(tp, fp, n_gt), rel=AP_RTOL,
                                                              abs=1e-15)
    a = torch.rand(37, 4)
    b = torch.rand(53, 4)
    a[:, 2:] += a[:, :2]
    b[:, 2:] += b[:, :2]
    got = um.calculate_iou_batch(a.cuda(), b.cuda()).cpu().numpy()
    assert np.array_equal(got, omet.calculate_iou_batch(a.numpy(), b.numpy()))
    assert float(um.calculate_iou(a[0].cuda(), b[0].cuda())) == float(omet.calculate_iou(a[0], b[0]))
