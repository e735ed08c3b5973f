"""yolomi — MI355X runtime for the YOLOv11 drop-in (ctypes over libyolomi.so).

Submodules
  _lib    loader + signatures of the C ABI (include/yolomi.h)
  post    decode + NMS postprocess
  graph   NHWC execution plan of the YOLOv11 graph (forward/backward)
  loss    fused assigner + CIoU/DFL/BCE loss kernels
"""
from ._lib import LIB_PATH, YolomiError, lib  # noqa: F401
