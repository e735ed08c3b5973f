#!/bin/bash
# round 6: the other BASELINE configs at HEAD — C4 (m@1280 bs16 training step) and C5 (s@640 inference bs 1 / 8 / 128)
set -o pipefail
O=gpurun_out/r06_extras
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --scale m --imgsz 1280 --batch 16 --steps 20 --warmup 3 --no-cpu-baseline > $O/c4_m1280.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
tail -c 300 $O/c4_m1280.json; echo
for rep in 1 2; do
  timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 128 --reps 200 --no-cpu-baseline > $O/c5_r$rep.json 2> $O/c5_r$rep.err || { tail -5 $O/c5_r$rep.err; exit 2; }
  echo "rep $rep $(python -c "
import json
for l in open('$O/c5_r$rep.json'):
    d = json.loads(l)
    if 'batch' in d: print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done
