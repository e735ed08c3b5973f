"""Data parallelism with the REAL plan at world size 2: two fresh processes share GPU 0
through gloo (YM_DIST_BACKEND / YM_DIST_DEVICE, yolomi/dist.py) and run tests/dp_worker.py.

* the synced gradient equals the mean of the two ranks' single-process gradients (fp32, 1e-6), on both
  ranks bit-identically, for the full bs2 plan and a partial bs1 last-batch plan;
* the first backward of a plan (one plain collective, hook attached) and the second (buckets issued from
  the backward hook on the side stream) give bit-identical gradients;
* train_yolo11_cuda.validate under DP (ValShard-style per-rank batches, detections gathered to rank 0,
  metrics broadcast) returns the same dict on both ranks, equal to validate() with dp=None over all
  batches in one process (losses 1e-6 relative; P / R / mAP identical up to 1e-9).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_world2_real_plan(tmp_path):
    env = dict(os.environ, YM_DIST_BACKEND="gloo", YM_DIST_DEVICE="0", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "tests" / "dp_worker.py"),
           str(tmp_path)]
    # own session: on a time-out the whole group (torchrun and both ranks) is killed, nothing keeps the GPU
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                            start_new_session=True)
    try:
        out, err = proc.communicate(timeout=110)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, 9)
        out, err = proc.communicate()
        pytest.fail(f"2-rank run timed out: {err[-4000:]}")
    assert proc.returncode == 0, (out[-3000:], err[-6000:])
    res = [json.loads((tmp_path / f"res_r{k}.json").read_text()) for k in range(2)]
    for case in ("full", "partial"):
        for k in range(2):
            info = res[k][case]
            assert info["hooked"] and info["buckets"] >= 2 and info["side_stream"], info
        loc = [torch.load(tmp_path / f"{case}_local_r{k}.pt", weights_only=True) for k in range(2)]
        g = {(it, k): torch.load(tmp_path / f"{case}_dp{it}_r{k}.pt", weights_only=True)
             for it in range(2) for k in range(2)}
        mean = (loc[0] + loc[1]) / 2
        for (it, k), t in g.items():
            assert torch.equal(t, g[(0, 0)]), (case, it, k)           # every rank, both iterations: identical
        err = float((g[(1, 0)].double() - mean.double()).norm() / mean.double().norm())
        assert err < 1e-6, (case, err)
    v0, v1 = res[0]["val_dp"], res[1]["val_dp"]
    assert v0 == v1
    w1 = res[0]["val_world1"]
    for k in ("loss", "box_loss", "cls_loss", "dfl_loss"):
        assert abs(v0[k] - w1[k]) <= 1e-6 * max(1.0, abs(w1[k])), (k, v0[k], w1[k])
    for k in ("precision", "recall", "mAP50", "mAP50-95"):
        assert abs(v0[k] - w1[k]) <= 1e-9, (k, v0[k], w1[k])
