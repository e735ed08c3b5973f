"""ctypes binding of libyolomi.so (the gfx950 C-ABI in include/yolomi.h).

The product path has no CPU fallback: if the library is missing or fails to
load, every entry point raises immediately.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_PKG = Path(__file__).resolve().parents[1]
LIB_PATH = Path(os.environ.get("YOLOMI_LIB", _PKG / "libyolomi.so"))

_c = ctypes
P, I64, I32, F32, SZ = _c.c_void_p, _c.c_int64, _c.c_int32, _c.c_float, _c.c_size_t

# name -> (restype, argtypes); must match include/yolomi.h
SIGNATURES = {
    "ym_last_error": (_c.c_char_p, []),
    "ym_version": (_c.c_int, []),
    "ym_iou_row": (_c.c_int, [P, P, I64, P, P]),
    "ym_nms_workspace_size": (SZ, [I64, I64]),
    "ym_decode_nms": (_c.c_int, [P, I64, I64, I64, I64, I64, F32, F32, F32, P, SZ, P, P, P, P, P, P]),
    "ym_nms": (_c.c_int, [P, P, I64, F32, P, SZ, P, P, P]),
}

_LIB = None


class YolomiError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise YolomiError(f"libyolomi not built: {LIB_PATH} missing (run `make -C yolo-scratch_amd/csrc`)")
        L = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def call(name: str, *args):
    st = getattr(lib(), name)(*args)
    if st != 0:
        raise YolomiError(f"{name} failed ({st}): {lib().ym_last_error().decode()}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise YolomiError("yolomi kernels run on the MI355X only: got a CPU tensor "
                              "(the CPU restatement lives in oracle/ and is test-only)")
