#!/bin/bash
# bs1 eval forward (small-grid eval path): wall per batch for graph x streams, then kernel traces
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_eval3
rm -rf $O; mkdir -p $O
for g in 0 1; do for s in 1 3; do
  YM_EVAL_GRAPH=$g YM_STREAMS=$s timeout -k 10 200 python -u $GRAFT_REPO_ROOT/tools/infer_bench.py --batches 1 --reps 100 --no-cpu-baseline > $O/g${g}_s${s}.json 2> $O/g${g}_s${s}.err || exit 1
  echo "graph=$g streams=$s $(python -c "import json; d=json.load(open('$O/g${g}_s${s}.json')); print(d['ms_per_batch'], d['value'])")"
done; done
cd /tmp && export TMPDIR=/tmp
for cfg in "1 1" "1 3" "0 3"; do set -- $cfg
  YM_EVAL_GRAPH=$1 YM_STREAMS=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t$1$2 -o trace -- python3 $GRAFT_REPO_ROOT/tools/infer_bench.py --batches 1 --reps 30 --no-cpu-baseline > $O/t$1$2.log 2>&1 || exit 1
  python3 $GRAFT_REPO_ROOT/tools/rocpd_summary.py $(find $O/t$1$2 -name "*.db" | head -1) --iter-kernel prep_weights_kernel --last 20 --top 40 > $O/t$1$2.txt || exit 1
  tail -1 $O/t$1$2.txt
done
