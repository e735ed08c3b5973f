#!/bin/bash
# round 5: eval small-grid K-split (ym_conv_fwd_eval workspace + eval_fold_kernel) — kernel parity, eval model tests,
# inference bench with the split at its default threshold vs off (ym_conv_set_eval_split=0), same box, interleaved;
# then a bs-1 kernel trace of the default
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_split
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_eval_conv.py tests/test_gpu_determinism.py tests/test_gpu_prep.py tests/test_gpu_model.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
for sp in 64 0 ${EXTRA_SPLIT:-}; do
  YM_LIB_SET="ym_conv_set_eval_split=$sp" timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 --reps 100 --no-cpu-baseline > $O/s${sp}_r$rep.json 2> $O/s${sp}_r$rep.err || exit 1
  echo "rep $rep split=$sp $(python -c "
import json
for l in open('$O/s${sp}_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t -o trace -- python3 $GRAFT_REPO_ROOT/tools/infer_bench.py --batches 1 --reps 30 --no-cpu-baseline > $O/t.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/rocpd_summary.py $(find $O/t -name "*.db" | head -1) --iter-kernel prep_weights_kernel --last 20 --top 40 --sequence > $O/t.txt || exit 1
rm -rf $O/t
tail -1 $O/t.txt
