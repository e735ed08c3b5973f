#!/bin/bash
# round 5: BatchNorm backward statistics + finalize in one launch on the 40x40 maps too (fold mode 2) — parity tests,
# then the training step A/B (default vs mode 2), interleaved, same box
set -o pipefail
O=gpurun_out/r05_bnfold
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bn.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2 3; do
  for mode in -1 2; do
    YM_LIB_SET="ym_bn_set_bwd_fold=$mode" timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 30 > $O/b_${mode}_$rep.json 2> $O/b_${mode}_$rep.err || { tail -5 $O/b_${mode}_$rep.err; exit 1; }
    echo "rep $rep mode $mode $(python -c "import json; d=json.load(open('$O/b_${mode}_$rep.json')); print(d['value'], d['ms_per_step'], 'bn', d['roofline_families']['bn']['ms_per_step'], d['roofline_families']['bn']['launch_groups'])")"
  done
done
