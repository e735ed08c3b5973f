"""Key-seeded weights — TEST INFRASTRUCTURE ONLY (never imported by the product path).

Fixtures must not carry 12-45 MB state_dicts, so every 4-D convolution weight
of a YOLOv11 state_dict is re-drawn from a generator seeded with crc32(key):

    W = randn(shape, Generator().manual_seed(crc32(key))) * sqrt(2 / fan_out)

which is the distribution the reference draws from with kaiming_normal_
(mode='fan_out', nonlinearity='relu') in
/root/reference/yolo_scratch_cuda/models/yolo11_model.py:177-182.  Everything
else (BN affine 1/0, running stats 0/0.97/1, Detect biases 1.0 and
log(1e-6)) is left exactly as the builder produced it
(yolo11_model.py:183-192, 194-229; yolo11_modules.py:268-274).
"""
from __future__ import annotations

import math
import zlib

import torch


def seeded_tensor(key: str, shape) -> torch.Tensor:
    g = torch.Generator().manual_seed(zlib.crc32(key.encode()))
    fan_out = shape[0]
    for s in shape[2:]:
        fan_out *= s
    return torch.randn(tuple(shape), generator=g, dtype=torch.float32) * math.sqrt(2.0 / fan_out)


def apply_seeded_weights(state: dict, prefix: str = "") -> dict:
    """In-place: overwrite every 4-D '*.weight' entry of a state_dict.  Keys are seeded without
    `prefix`, so a block's parameters held under 'blk.' in the oracle draw the same values as the
    standalone module's state_dict (keys 'cv1.conv.weight', ...)."""
    for k, v in state.items():
        if k.endswith(".weight") and v.dim() == 4:
            v.copy_(seeded_tensor(k[len(prefix):] if k.startswith(prefix) else k, v.shape))
    return state
