import sys, ctypes, os
sys.path.insert(0, __import__('os').environ.get('GRAFT_REPO_ROOT', '/root/repo')); sys.path.insert(0, __import__('os').environ.get('GRAFT_REPO_ROOT', '/root/repo') + '/yolo-scratch_amd')
os.environ.setdefault("YM_NMS_STAMPS", "1")
import torch
from datasets.synthetic import synth_eval_preds
from yolomi import post as ypost
from yolomi._lib import lib
pd = synth_eval_preds(1, 8400, seed=8).cuda()
for _ in range(3):
    ypost.decode_nms(pd, 640, 0.25, 0.45)
torch.cuda.synchronize()
a = (ctypes.c_ulonglong * 4)()
lib().ym_debug_nms_stamps(a)
print("cycles per segment (wave scan: group start, chunks, group end, epilogue | triangle scan: load issue, reduce, resolve, store):", list(a), "sum", sum(a))
