#!/bin/bash
# round 5: the inference bench (configs[4], bs 1 / 8 / 128), two runs on one box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_infer
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 128 --reps 200 ${CPU_BASE:---no-cpu-baseline} > $O/r$rep.json 2> $O/r$rep.err || exit 1
  echo "rep $rep $(python -c "
import json
for l in open('$O/r$rep.json'):
    d = json.loads(l)
    if 'batch' in d: print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done
