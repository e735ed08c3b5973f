"""GPU parity of the decode + NMS postprocess against the reference goldens and
the C oracle: keep lists and boxes bit-exact (tie-free inputs)."""
import numpy as np
import pytest
import torch

from oracle import post as op

pytestmark = pytest.mark.gpu


def test_iou_row_bitexact(golden):
    from yolomi import post
    d = golden("nms.npz")
    out = post.iou_row(torch.from_numpy(d["iou_b1"]).cuda(), torch.from_numpy(d["iou_b2"]).cuda()).cpu().numpy()
    np.testing.assert_array_equal(out.view(np.uint32), d["iou_out"].astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("n", [0, 1, 2, 100, 1000, 6700])
def test_nms_keep_bitexact(golden, n):
    from yolomi import post
    d = golden("nms.npz")
    keep = post.nms(torch.from_numpy(d[f"n{n}_boxes"]).cuda(), torch.from_numpy(d[f"n{n}_scores"]).cuda(), 0.45)
    np.testing.assert_array_equal(keep.cpu().numpy(), d[f"n{n}_keep"])


@pytest.mark.parametrize("kind", ["am", "lit"])
def test_decode_nms_bitexact(golden, kind):
    import train_yolo11_cuda as T
    d = golden("decode.npz")
    pred = torch.from_numpy(d[f"{kind}_in"]).cuda()
    out = T.decode_predictions_for_metrics(pred, 640, 0.25, 0.45, pred.device)
    counts = np.asarray([len(o["scores"]) for o in out])
    np.testing.assert_array_equal(counts, d[f"{kind}_counts"])
    np.testing.assert_array_equal(torch.cat([o["boxes"] for o in out]).cpu().numpy(), d[f"{kind}_boxes"])
    np.testing.assert_array_equal(torch.cat([o["scores"] for o in out]).cpu().numpy(), d[f"{kind}_scores"])
    np.testing.assert_array_equal(torch.cat([o["labels"] for o in out]).cpu().numpy(), d[f"{kind}_labels"])


@pytest.mark.parametrize("seed,B,N", [(5, 1, 8400), (6, 8, 8400), (7, 3, 17)])
def test_decode_nms_strided_view_vs_oracle(seed, B, N):
    """The anchor-major VIEW of a (B, 4+nc, A) tensor (what the eval loop passes: y.transpose(1, 2)) decodes in place
    (ym_decode_nms_strided, elements A apart) to the oracle's result on the same rows, bit-exact."""
    import train_yolo11_cuda as T
    from datasets.synthetic import synth_eval_preds
    pred = synth_eval_preds(B, N, seed=seed)
    ref = op.decode(pred.numpy(), 640, 0.25, 0.45)
    view = pred.cuda().transpose(1, 2).contiguous().transpose(1, 2)
    assert view.stride(-1) == N
    out = T.decode_predictions_for_metrics(view, 640, 0.25, 0.45, torch.device("cuda"))
    for (rb, rs, rl), o in zip(ref, out):
        np.testing.assert_array_equal(o["scores"].cpu().numpy(), rs)
        np.testing.assert_array_equal(o["boxes"].cpu().numpy(), rb)
        np.testing.assert_array_equal(o["labels"].cpu().numpy(), rl)


@pytest.mark.parametrize("seed,B,N", [(1, 4, 8400), (2, 128, 8400), (3, 2, 33600), (4, 3, 17)])
def test_decode_nms_vs_oracle_random(seed, B, N):
    """Fresh synthetic inputs (incl. the 1280² anchor count) against the C oracle."""
    import train_yolo11_cuda as T
    from datasets.synthetic import synth_eval_preds
    pred = synth_eval_preds(B, N, seed=seed)
    ref = op.decode(pred.numpy(), 640, 0.25, 0.45)
    out = T.decode_predictions_for_metrics(pred.cuda(), 640, 0.25, 0.45, torch.device("cuda"))
    for (rb, rs, rl), o in zip(ref, out):
        np.testing.assert_array_equal(o["scores"].cpu().numpy(), rs)
        np.testing.assert_array_equal(o["boxes"].cpu().numpy(), rb)
        np.testing.assert_array_equal(o["labels"].cpu().numpy(), rl)
