#!/bin/bash
# bs1 eval forward: graph vs eager x 1 / 3 scheduler streams, then a kernel trace of the eager 3-stream run
set -o pipefail
O=gpurun_out/r05_eval2
mkdir -p $O
for g in 0 1; do for s in 1 3; do
  YM_EVAL_GRAPH=$g YM_STREAMS=$s timeout -k 10 200 python -u tools/infer_bench.py --batches 1 --reps 100 --no-cpu-baseline > $O/g${g}_s${s}.json 2> $O/g${g}_s${s}.err || exit 1
  echo "graph=$g streams=$s $(python -c "import json,sys; d=json.load(open('$O/g${g}_s${s}.json')); print(d['ms_per_batch'], d['value'])")"
done; done
cd /tmp && export TMPDIR=/tmp
YM_EVAL_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o trace -- python3 $GRAFT_REPO_ROOT/tools/infer_bench.py --batches 1 --reps 30 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
echo done
