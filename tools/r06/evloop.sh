#!/bin/bash
# round 6: the nested loop form (LP 2) in conv_pipe's eval instance — eval parity tests with the shipping library, then
# inference bs 1 / 8 / 128 with the flat (0) and nested (2) forms interleaved (measurement library, YM_LIB_SET)
set -o pipefail
O=gpurun_out/r06_evloop
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_eval_conv.py tests/test_gpu_c5_eval.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export YOLOMI_LIB=$PWD/yolo-scratch_amd/libyolomi_exp.so
for rep in 1 2; do for v in 0 2; do
  YM_LIB_SET="ym_conv_set_pipe_eval_loop=$v" timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 128 --reps 200 --no-cpu-baseline > $O/v${v}_r$rep.json 2> $O/v${v}_r$rep.err || { tail -5 $O/v${v}_r$rep.err; exit 2; }
  echo "loop $v rep $rep $(python -c "
import json
for l in open('$O/v${v}_r$rep.json'):
    d = json.loads(l)
    if 'batch' in d: print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
