"""Data path: the reference's crater loader and batch-dict contract, plus synthetic batches.

CraterDatasetCUDA mirrors /root/reference/yolo_scratch_cuda/datasets/crater_dataset_cuda.py:26-286
(decode in the workers, stretch-resize on the GPU: datasets/crater.py); collate_fn_cuda mirrors
:289-346; prepare_batch is the device transfer of train_yolo11_cuda.py:43-45.
"""
from .collate import collate_fn_cuda  # noqa: F401
from .crater import CraterDatasetCUDA, max_gt_count, prepare_batch, resize_batch  # noqa: F401

collate_fn = collate_fn_cuda
CraterDatasetYOLO = CraterDatasetCUDA

__all__ = ["CraterDatasetCUDA", "CraterDatasetYOLO", "collate_fn_cuda", "collate_fn", "prepare_batch"]
