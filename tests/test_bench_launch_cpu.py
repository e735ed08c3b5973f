"""bench.py's N-rank launcher (BASELINE metric: img/s at 1/2/4/8 GPUs): `python bench.py --gpus N` run
directly starts N ranks itself (torchrun as a child process of a parent that never touches the GPU), and a
rank refuses to report when the job's size differs from --gpus.  CPU only: the ranks run the launcher check
mode (YM_BENCH_RANKS_ONLY=1: init over gloo, one all-reduce of ones, rank 0 prints the count)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_needs_launch_rules():
    assert bench.needs_launch(2, {})
    assert bench.needs_launch(8, {"MASTER_ADDR": "127.0.0.1"})
    assert not bench.needs_launch(1, {})
    assert not bench.needs_launch(2, {"WORLD_SIZE": "2", "RANK": "0"})     # already a torchrun rank
    cmd = bench.launch_cmd(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(YM_BENCH_RANKS_ONLY="1", MASTER_ADDR="127.0.0.1", **(extra_env or {}))
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], env=env, capture_output=True, text=True,
                          timeout=240)


def test_gpus2_starts_two_ranks():
    r = _run(["--gpus", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout                     # rank 0 alone prints
    assert json.loads(lines[0]) == {"n_gpus": 2, "ranks_seen": 2}


def test_world_mismatch_fails_loudly():
    # a 2-rank job asked to report 3 GPUs: every rank exits non-zero instead of reporting 2 as 3
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(YM_BENCH_RANKS_ONLY="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={bench.free_port()}", str(ROOT / "bench.py"),
                        "--gpus", "3"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert "--gpus 3 but this job has 2 rank(s)" in r.stderr
