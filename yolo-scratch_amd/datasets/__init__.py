"""Data path: the reference's batch-dict contract plus synthetic batches.

collate_fn_cuda mirrors /root/reference/yolo_scratch_cuda/datasets/crater_dataset_cuda.py:289-346.
"""
from .collate import collate_fn_cuda, CraterDatasetCUDA  # noqa: F401

collate_fn = collate_fn_cuda
CraterDatasetYOLO = CraterDatasetCUDA

__all__ = ["CraterDatasetCUDA", "collate_fn_cuda", "collate_fn"]
