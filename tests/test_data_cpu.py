"""Crater data path on the CPU: annotation parsing, targets, decode and collate packing of
datasets/crater.py against the oracle restatement of the reference loader (oracle/data.py,
crater_dataset_cuda.py:77-124, 162-186, 253-279, 289-346), and OpenCV INTER_LINEAR sanity checks
of that restatement (parity vs cv2 itself is unpinned: no cv2 in this image)."""
import functools

import numpy as np
import torch

from data_cases import make_dataset


def test_annotations_targets_and_decode(tmp_path):
    from oracle import data as od
    from datasets import CraterDatasetCUDA
    make_dataset(tmp_path)
    ds = CraterDatasetCUDA(tmp_path, img_size=640)
    ref = od.load_annotations(tmp_path)
    assert len(ds) == len(ref) == 5
    for i, (path, anns) in enumerate(ref):
        s = ds.samples[i]
        assert s["img_path"] == path
        assert [(a["cx"], a["cy"], a["w"], a["h"], a["class"]) for a in s["annotations"]] == list(anns)
        img, boxes, labels, idx = ds[i]
        assert idx == i and img.dtype == torch.uint8 and img.shape[0] == 1
        h0, w0 = img.shape[1:]
        rb, rl = od.targets(anns, h0, w0)
        assert np.array_equal(boxes.numpy(), rb) and np.array_equal(labels.numpy(), rl)
        from PIL import Image
        with Image.open(path) as im:
            a = np.asarray(im)
        want = od.gray_from_rgb(a) if a.ndim == 3 else a
        assert np.array_equal(img[0].numpy(), want)


def test_collate_packs_raw_images(tmp_path):
    from datasets import CraterDatasetCUDA, collate_fn_cuda
    make_dataset(tmp_path)
    ds = CraterDatasetCUDA(tmp_path, img_size=320)
    items = [ds[i] for i in range(len(ds))]
    b = functools.partial(collate_fn_cuda, img_size=320)(items)
    assert b["img_size"] == 320 and b["img_meta"].shape == (5, 3)
    off = 0
    for (img, boxes, labels, _), m in zip(items, b["img_meta"].tolist()):
        h, w = img.shape[1:]
        assert m == [off, h, w]
        assert torch.equal(b["img_u8"][off:off + h * w], img.reshape(-1))
        off += h * w
    n = sum(len(it[1]) for it in items)
    assert b["batch_idx"].shape == (n,) and b["cls"].shape == (n, 1) and b["bboxes"].shape == (n, 4)
    assert float(b["bboxes"].min()) >= 0.0 and float(b["bboxes"].max()) <= 1.0


def test_resize_restatement_sanity():
    from oracle.data import resize_linear_u8
    # the commonly quoted cv2.resize(np.uint8([[0, 255]]), (4, 1), interpolation=INTER_LINEAR) result
    assert resize_linear_u8(np.uint8([[0, 255]]), 4)[0].tolist() == [0, 64, 191, 255]
    # identity at the target size, constants stay constant, exact 2x down-sampling of 2x2 blocks
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (64, 64), dtype=np.uint8)
    assert np.array_equal(resize_linear_u8(a, 64), a)
    assert (resize_linear_u8(np.full((37, 91), 200, np.uint8), 50) == 200).all()
    blocks = a.reshape(32, 2, 32, 2).astype(np.int64)
    r = resize_linear_u8(a, 32).astype(np.int64)
    assert np.abs(r - blocks.mean((1, 3))).max() <= 1


def test_prepare_batch_records_max_gt_on_host():
    """prepare_batch counts the max GTs per image on the host (the loss then needs no device sync)."""
    import torch
    from datasets import max_gt_count, prepare_batch
    from datasets.synthetic import synth_batch
    b = synth_batch(6, 64, seed=5)
    want = int(torch.bincount(b["batch_idx"].long(), minlength=6).max())
    out = prepare_batch(b, "cpu")
    assert out["max_gt"] == want == max_gt_count(b["batch_idx"])
    assert max_gt_count(torch.zeros(0)) == 0
