#!/bin/bash
# round 5: eval-mode Conv blocks in one launch (ym_conv_fwd_eval) — kernel parity, eval model tests, inference bench
# with them on (default) and off (YM_EVAL_FUSE=0), same box, interleaved
set -o pipefail
O=gpurun_out/r05_eval
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_eval_conv.py tests/test_gpu_determinism.py tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_boundary.py tests/test_gpu_train_entry.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
for f in 1 0; do
  YM_EVAL_FUSE=$f timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 128 --reps 100 --no-cpu-baseline > $O/f${f}_r$rep.json 2> $O/f${f}_r$rep.err || exit 1
  echo "rep $rep fuse=$f $(python -c "
import json
for l in open('$O/f${f}_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
