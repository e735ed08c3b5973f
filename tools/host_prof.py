"""Host-side profile (cProfile) of the eval forward at bs1 — where the Python enqueue time goes; with "e2e" as the
second argument, of the inference bench's batch (forward + decode_predictions_for_metrics, which synchronises).
usage: python tools/host_prof.py [reps] [e2e]"""
import cProfile
import pstats
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd")]
import torch
import yaml
from models import build_yolo11

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
e2e = len(sys.argv) > 2 and sys.argv[2] == "e2e"
cfg = yaml.safe_load((ROOT / "yolo-scratch_amd" / "configs" / "yolo11n_crater.yaml").read_text())
cfg["scale"] = "s"
m = build_yolo11(cfg, ch=1, nc=5).cuda().eval()
img = torch.rand(1, 1, 640, 640, device="cuda")
with torch.no_grad():
    for _ in range(3):
        m(img)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        m(img)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / reps:.3f} ms/forward, wall {1e3 * (t2 - t0) / reps:.3f} ms/forward")
    import train_yolo11_cuda as T

    def batch():
        y = m(img)
        if e2e:
            T.decode_predictions_for_metrics(y[0].transpose(1, 2), 640, 0.25, 0.45, img.device)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(reps):
        batch()
    pr.disable()
    torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
