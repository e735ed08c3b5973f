"""GPU data path: ym_resize_linear_u8 bit-exact against the OpenCV INTER_LINEAR restatement
(oracle/data.py), and dataset -> collate -> prepare_batch producing the reference's batch dict
(img (B, 1, S, S) fp32, targets) exactly as the oracle loader would."""
import functools

import numpy as np
import pytest
import torch

from data_cases import make_dataset

pytestmark = pytest.mark.gpu

SIZES = [(480, 640), (700, 517), (640, 640), (1, 2), (3, 1000), (1024, 1024), (333, 333), (81, 1279)]


@pytest.mark.parametrize("S", [640, 320, 1280])
def test_resize_kernel_bitexact(S):
    from oracle.data import resize_linear_u8
    from datasets.crater import pack_images, resize_batch
    rng = np.random.default_rng(S)
    ims = [rng.integers(0, 256, hw, dtype=np.uint8) for hw in SIZES]
    ims.append(np.full((17, 23), 255, np.uint8))
    ims.append(np.zeros((S, S), np.uint8) + np.arange(S, dtype=np.uint8)[None])   # already S x S
    p = pack_images([torch.from_numpy(a).unsqueeze(0) for a in ims], S)
    out = resize_batch(p["img_u8"].cuda(), p["img_meta"].cuda(), S).cpu()
    for i, a in enumerate(ims):
        want = resize_linear_u8(a, S).astype(np.float32) / np.float32(255.0)
        assert np.array_equal(out[i, 0].numpy(), want), (i, a.shape)


def test_dataset_to_device_batch(tmp_path):
    from oracle import data as od
    from datasets import CraterDatasetCUDA, collate_fn_cuda, prepare_batch
    make_dataset(tmp_path, seed=3)
    ds = CraterDatasetCUDA(tmp_path, img_size=640)
    dl = torch.utils.data.DataLoader(ds, batch_size=3, shuffle=False,
                                     collate_fn=functools.partial(collate_fn_cuda, img_size=640))
    ref = od.load_annotations(tmp_path)
    seen = 0
    for b in dl:
        d = prepare_batch(b, torch.device("cuda"))
        assert set(d) == {"img", "batch_idx", "cls", "bboxes", "max_gt"}
        assert d["max_gt"] == int(torch.bincount(d["batch_idx"].long().cpu()).max()) if len(d["batch_idx"]) else 0
        assert d["img"].shape == (len(d["img"]), 1, 640, 640) and d["img"].dtype == torch.float32
        for j in range(d["img"].shape[0]):
            path, anns = ref[seen + j]
            from PIL import Image
            with Image.open(path) as im:
                a = np.asarray(im)
            a = od.gray_from_rgb(a) if a.ndim == 3 else a
            assert np.array_equal(d["img"][j].cpu().numpy(), od.image_tensor(a, 640))
            rb, rl = od.targets(anns, *a.shape)
            m = (d["batch_idx"] == j).cpu()
            c, wh = rb[:, :2], rb[:, 2:]
            xyxy = np.clip(np.concatenate([c - wh / 2, c + wh / 2], 1), 0, 1)
            assert np.allclose(d["bboxes"].cpu()[m].numpy(), xyxy, rtol=0, atol=1e-7)
            assert np.array_equal(d["cls"].cpu()[m].reshape(-1).numpy(), rl)
        seen += d["img"].shape[0]
    assert seen == len(ds)
