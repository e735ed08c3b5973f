#!/bin/bash
# round 5: eval forward replayed as a HIP graph on one stream — determinism / eval tests, then the inference bench
# (graph default vs eager three streams vs graph three streams), same box
set -o pipefail
O=gpurun_out/r05_eval
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_determinism.py tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_boundary.py tests/test_gpu_train_entry.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
for v in "1 -" "0 3" "1 3"; do set -- $v
  if [ "$2" = "-" ]; then unset YM_STREAMS; else export YM_STREAMS=$2; fi
  YM_EVAL_GRAPH=$1 timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 128 --reps 100 --no-cpu-baseline > $O/g$1_s$2_r$rep.json 2> $O/g$1_s$2_r$rep.err || exit 1
  echo "rep $rep graph=$1 streams=$2 $(python -c "
import json
for l in open('$O/g$1_s$2_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
unset YM_STREAMS
