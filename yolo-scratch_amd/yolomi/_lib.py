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

INT, F64 = _c.c_int, _c.c_double


class ConvDesc(ctypes.Structure):
    """ym_conv_desc (include/yolomi.h)."""
    _fields_ = [("n", I32), ("h", I32), ("w", I32), ("cin", I32), ("oh", I32), ("ow", I32), ("cout", I32),
                ("k", I32), ("stride", I32), ("pad", I32), ("x_bs", I64), ("x_ld", I64), ("y_bs", I64),
                ("y_ld", I64), ("out_f32", I32), ("accumulate", I32)]


class AdamWEntry(ctypes.Structure):
    """ym_adamw_entry (include/yolomi.h)."""
    _fields_ = [("p", P), ("g", P), ("m", P), ("v", P), ("offset", I64), ("n", I64)]


class WPrepEntry(ctypes.Structure):
    """ym_wprep_entry (include/yolomi.h)."""
    _fields_ = [("src", P), ("dst_fwd", P), ("dst_t", P), ("elem_offset", I64), ("cout", I32), ("cin", I32),
                ("kh", I32), ("kw", I32), ("cout_t", I32)]


class BnEvalEntry(ctypes.Structure):
    """ym_bn_eval_entry (include/yolomi.h)."""
    _fields_ = [("gamma", P), ("beta", P), ("running_mean", P), ("running_var", P), ("scale", P), ("shift", P),
                ("c", I32), ("eps", _c.c_float)]


class BnFold(ctypes.Structure):
    """ym_bn_fold (include/yolomi.h)."""
    _fields_ = [("gamma", P), ("beta", P), ("running_mean", P), ("running_var", P), ("num_batches_tracked", P),
                ("scale", P), ("shift", P), ("mean", P), ("rstd", P), ("workspace", P), ("count", F64),
                ("momentum", _c.c_float), ("eps", _c.c_float)]


R = _c.c_int
# name -> (restype, argtypes); must match include/yolomi.h + include/yolomi_experimental.h (its YM_EXPERIMENTS block
# excepted: the measurement library's)
SIGNATURES = {
    "ym_last_error": (_c.c_char_p, []),
    "ym_version": (R, []),
    "ym_policy_generation": (_c.c_uint, []),
    "ym_iou_row": (R, [P, P, I64, P, P]),
    "ym_nms_workspace_size": (SZ, [I64, I64]),
    "ym_decode_nms": (R, [P, I64, I64, I64, I64, I64, F32, F32, F32, P, SZ, P, P, P, P, P, P]),
    "ym_decode_nms_strided": (R, [P, I64, I64, I64, I64, I64, I64, F32, F32, F32, P, SZ, P, P, P, P, P, P]),
    "ym_nms": (R, [P, P, I64, F32, P, SZ, P, P, P]),
    "ym_conv_stat_blocks": (R, [I64, INT]),
    "ym_conv_fwd_stat_rows": (R, [P]),
    "ym_conv_algo": (R, [P, INT]),
    "ym_conv_kernel": (R, [P, INT, P, INT]),
    "ym_conv_set_select_batch": (R, [INT]),
    "ym_conv_set_halo": (R, [INT]),
    "ym_conv_set_pipe": (R, [INT]),
    "ym_conv_set_direct": (R, [INT]),
    "ym_conv_set_hpipe": (R, [INT]),
    "ym_conv_fwd": (R, [P, P, P, P, P, P, P, P]),
    "ym_conv_dgrad": (R, [P, P, P, P, P]),
    "ym_conv_wgrad_workspace_size": (SZ, [P]),
    "ym_wgrad_set_target": (R, [INT]),
    "ym_conv_wgrad": (R, [P, P, P, P, SZ, P, INT, P]),
    "ym_conv_first_fwd": (R, [P, P, P, P, P, INT, INT, INT, INT, INT, INT, INT, INT, INT, INT, P]),
    "ym_conv_first_fwd_eval": (R, [P, P, P, P, INT, P, I64, I64, INT, INT, INT, INT, INT, INT, INT, INT, INT, P]),
    "ym_stem_bwd_wgrad_workspace_size": (SZ, [INT]),
    "ym_stem_bwd_wgrad_stored": (R, [P, I64, I64, P, P, P, P, P, P, SZ, INT, INT, INT, INT, INT, INT, INT, INT, P]),
    "ym_conv_first_wgrad_workspace_size": (SZ, [INT, INT]),
    "ym_conv_first_wgrad": (R, [P, P, P, INT, INT, INT, INT, INT, INT, INT, INT, INT, P, SZ, P]),
    "ym_dw3x3_fwd": (R, [P, I64, I64, INT, INT, INT, P, P, P, P, INT, INT, INT, INT, INT, P]),
    "ym_dw3x3_fwd_eval": (R, [P, I64, I64, INT, INT, INT, P, P, P, INT, P, I64, I64, P, I64, I64, INT, INT, INT, INT,
                              P]),
    "ym_dw3x3_bwd_workspace_size": (SZ, [INT]),
    "ym_dw3x3_bwd": (R, [P, I64, I64, INT, INT, INT, P, P, P, I64, I64, P, INT, INT, INT, INT, INT, P, SZ, P]),
    "ym_prep_weights": (R, [P, INT, I64, P]),
    "ym_prep_weights_fwd": (R, [P, INT, I64, P]),
    "ym_bn_workspace_size": (SZ, [INT]),
    "ym_conv_fwd_bn_fused": (R, [P]),
    "ym_conv_fwd_bn": (R, [P, P, P, P, P, P, P, P]),
    "ym_conv_set_fold": (R, [INT]),
    "ym_conv_fwd_eval_ok": (R, [P]),
    "ym_conv_set_eval_cfg": (R, [INT]),
    "ym_conv_set_eval_narrow": (R, [INT]),
    "ym_conv_fwd_eval_workspace_size": (SZ, [P]),
    "ym_conv_set_eval_split": (R, [INT]),
    "ym_conv_set_eval_split_nk": (R, [INT]),
    "ym_conv_set_eval_pipe": (R, [INT]),
    "ym_conv_set_eval_route": (R, [INT]),
    "ym_conv_set_eval_gemm_tiles": (R, [INT]),
    "ym_conv_fwd_eval": (R, [P, P, P, P, P, INT, P, I64, I64, P, P, SZ, P]),
    "ym_bn_finalize": (R, [P, P, INT, INT, F64, P, P, P, P, P, F32, F32, P, P, P, P, P, P]),
    "ym_bn_eval_coeff": (R, [INT, P, P, P, P, F32, P, P, P]),
    "ym_bn_eval_coeff_batch": (R, [P, INT, P]),
    "ym_bn_apply": (R, [P, I64, INT, INT, P, P, INT, P, I64, I64, P, I64, I64, P, P]),
    "ym_bn_bwd_blocks": (R, [I64, INT]),
    "ym_bn_bwd_reduce": (R, [P, I64, I64, P, I64, INT, INT, P, P, P, P, INT, P, P, P]),
    "ym_bn_bwd_finalize": (R, [P, P, INT, INT, F64, P, P, P, P, INT, P, P, P]),
    "ym_bn_bwd_fold_ok": (R, [I64, INT]),
    "ym_bn_bwd_reduce_fold": (R, [P, I64, I64, P, I64, INT, INT, P, P, P, P, INT, P, P, P, P, P, INT, P, P, P]),
    "ym_bn_set_bwd_fold": (R, [INT]),
    "ym_bn_bwd_apply": (R, [P, I64, I64, P, I64, INT, INT, P, P, P, P, INT, P, P, P]),
    "ym_bn_bwd_apply_res": (R, [P, I64, I64, P, I64, INT, INT, P, P, P, P, INT, P, P, P, I64, I64, INT, P]),
    "ym_sppf_supported": (R, [INT, INT, INT]),
    "ym_sppf_fwd": (R, [P, P, P, P, P, I64, I64, P, INT, INT, INT, INT, P]),
    "ym_sppf_bwd": (R, [P, P, P, P, I64, I64, P, I64, I64, INT, P, INT, INT, INT, INT, P]),
    "ym_maxpool5_f32_fwd": (R, [P, P, P, P, I64, I64, INT, INT, INT, INT, P]),
    "ym_maxpool5_f32_bwd": (R, [P, P, P, I64, I64, P, P, I64, I64, INT, INT, INT, INT, INT, P]),
    "ym_upsample2_fwd": (R, [P, I64, I64, P, I64, I64, INT, INT, INT, INT, P]),
    "ym_upsample2_bwd": (R, [P, I64, I64, P, I64, I64, INT, INT, INT, INT, INT, P]),
    "ym_view_to_f32": (R, [P, I64, I64, P, I64, INT, INT, P]),
    "ym_f32_to_view": (R, [P, P, I64, I64, I64, INT, INT, INT, P]),
    "ym_view_axpy": (R, [P, I64, I64, P, I64, I64, I64, INT, INT, INT, INT, P]),
    "ym_head_grad_workspace_size": (SZ, []),
    "ym_head_grad": (R, [P, I64, I64, INT, I64, INT, P, P, P, P, P, SZ, P]),
    "ym_attn_fwd": (R, [P, I64, I64, INT, INT, INT, INT, INT, F32, P, I64, I64, P, P]),
    "ym_attn_workspace_size": (SZ, [INT, INT, INT]),
    "ym_attn_bwd": (R, [P, I64, I64, P, I64, I64, P, I64, I64, P, INT, INT, INT, F32, P, P, I64, I64, INT, INT, INT,
                        P]),
    "ym_loss_workspace_size": (SZ, [I64, I64, INT]),
    "ym_loss_fwd": (R, [P, I64, I64, INT, INT, P, P, P, P, P, P, I64, INT, F32, F32, P, SZ, P, P, P, P, P]),
    "ym_loss_bwd": (R, [P, I64, I64, INT, INT, P, P, P, INT, P, SZ, P, P, P, P, P, P]),
    "ym_loss_assignment": (R, [P, I64, I64, INT, P, P, P]),
    "ym_detect_decode": (R, [P, I64, I64, INT, INT, P, P, P, P, P, P]),
    "ym_dfl_fwd": (R, [P, I64, I64, INT, P, P, P]),
    "ym_dfl_bwd": (R, [P, I64, I64, INT, P, P, P, P]),
    "ym_tal_assign_workspace_size": (SZ, [I64, I64, INT]),
    "ym_tal_assign": (R, [P, P, P, P, P, P, I64, I64, INT, INT, F32, F32, F32, P, SZ, P, P, P, P, P, P]),
    "ym_bbox_loss_workspace_size": (SZ, [I64, I64]),
    "ym_bbox_loss_fwd": (R, [P, P, P, P, P, P, P, I64, I64, INT, P, SZ, P, P]),
    "ym_bbox_loss_bwd": (R, [P, P, P, P, P, P, P, I64, I64, INT, P, P, P, P]),
    "ym_copy2d": (R, [P, I64, P, I64, I64, I64, P]),
    "ym_eval_workspace_size": (SZ, [I64, I64, INT]),
    "ym_eval_detections": (R, [P, P, P, P, P, I64, I64, I64, I64, P, INT, INT, INT, F32, P, SZ, P, P]),
    "ym_eval_ap": (R, [P, P, I64, I64, P, SZ, P, P]),
    "ym_iou_matrix": (R, [P, P, I64, I64, P, P]),
    "ym_resize_linear_u8": (R, [P, P, INT, INT, P, P]),
    "ym_grad_norm_blocks": (R, [I64]),
    "ym_grad_norm": (R, [P, INT, I64, P, P, P]),
    "ym_adamw": (R, [P, INT, I64, F64, F64, F64, F64, F64, I64, F32, P, P]),
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
            # a library named by YOLOMI_LIB (an earlier build, for A/B runs) may predate later entry points
            fn = getattr(L, name, None) if "YOLOMI_LIB" in os.environ else getattr(L, name)
            if fn is None:
                continue
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
