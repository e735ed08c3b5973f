"""Postprocess-only loop for a kernel trace: ym_decode_nms on the SURVEY §8(d) workload at batch B
(default 1), --reps calls.  usage: rocprofv3 --kernel-trace ... -- python3 tools/post_prof.py [B reps]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yolo-scratch_amd")]
import torch
from datasets.synthetic import synth_eval_preds
from yolomi import post as ypost

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
pd = synth_eval_preds(B, 8400, seed=7 + B).cuda()
for _ in range(reps):
    ypost.decode_nms(pd, 640, 0.25, 0.45)
torch.cuda.synchronize()
