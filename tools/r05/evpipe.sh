#!/bin/bash
# round 5: the pipelined forward's eval instance — eval parity tests, then the inference bench with it on (default) and
# off (ym_conv_set_eval_pipe=0), bs 1 / 8 / 128, same box, interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_evpipe
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eval_conv.py tests/test_gpu_determinism.py tests/test_gpu_model.py > $O/test.log 2>&1 || { grep -E "^(FAILED|E )" $O/test.log | head -20; tail -5 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do for v in 1 0; do
  YM_LIB_SET="ym_conv_set_eval_pipe=$v" timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 128 --reps 100 --no-cpu-baseline > $O/p${v}_r$rep.json 2> $O/p${v}_r$rep.err || exit 1
  echo "rep $rep eval_pipe=$v $(python -c "
import json
for l in open('$O/p${v}_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
