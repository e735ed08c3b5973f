#!/bin/bash
# round 5: kernel trace summary of the bs-128 eval forward (inference bench, graph replay)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_bs8
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t -o trace -- python3 $GRAFT_REPO_ROOT/tools/infer_bench.py --batches 8 --reps 30 --no-cpu-baseline > $O/t.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/rocpd_summary.py $(find $O/t -name "*.db" | head -1) --iter-kernel prep_weights_kernel --last 20 --top 30 --sequence > $O/t.txt || exit 1
rm -rf $O/t
head -32 $O/t.txt
