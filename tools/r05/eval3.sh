#!/bin/bash
# bs1 eval forward (shipped default: one-launch Conv blocks, single-stream graph): kernel trace summary per forward
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_eval3
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t -o trace -- python3 $GRAFT_REPO_ROOT/tools/infer_bench.py --batches 1 --reps 30 --no-cpu-baseline > $O/t.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/rocpd_summary.py $(find $O/t -name "*.db" | head -1) --iter-kernel prep_weights_kernel --last 20 --top 40 --sequence > $O/t.txt || exit 1
rm -rf $O/t
tail -3 $O/t.txt
timeout -k 10 200 python3 -u $GRAFT_REPO_ROOT/tools/eval_bs1_probe.py --reps 200 > $O/probe.txt 2>&1 && cat $O/probe.txt
