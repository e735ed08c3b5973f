import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "yolo-scratch_amd"
GOLDEN = ROOT / "tests" / "golden"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long CPU test")
    # parity runs of a non-default library policy: YM_LIB_SET="ym_conv_set_eval_cfg=2 ..." calls those process-wide
    # setters (include/yolomi.h) before any test (unset in the driver's runs)
    if os.environ.get("YM_LIB_SET"):
        from yolomi._lib import lib
        for kv in os.environ["YM_LIB_SET"].split():
            name, val = kv.split("=")
            getattr(lib(), name)(int(val))


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)
    return load


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
