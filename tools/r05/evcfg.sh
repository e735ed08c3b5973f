#!/bin/bash
# eval GEMM stage / ring configurations (ym_conv_set_eval_cfg 0 / 1 / 2), bs 1 / 8, same box, interleaved; parity first
set -o pipefail
O=gpurun_out/r05_evcfg
rm -rf $O; mkdir -p $O
for c in 0 1 2; do
  YM_LIB_SET="ym_conv_set_eval_cfg=$c" timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_eval_conv.py > $O/test_$c.log 2>&1 || { tail -20 $O/test_$c.log; exit 1; }
done
tail -1 $O/test_2.log
for rep in 1 2; do for c in 0 1 2; do
  YM_LIB_SET="ym_conv_set_eval_cfg=$c" timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 --reps 100 --no-cpu-baseline > $O/c${c}_r$rep.json 2> $O/c${c}_r$rep.err || exit 1
  echo "rep $rep cfg=$c $(python -c "
import json
for l in open('$O/c${c}_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
