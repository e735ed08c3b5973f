#!/bin/bash
# round 5: kernel trace of a few bench steps -> the forward/loss/backward transition window of the middle step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_window
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 1
KT=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_window.py $KT ${FROM:-6.3} ${TO:-7.6} > $O/window.txt || exit 1
python3 $GRAFT_REPO_ROOT/tools/trace_streams.py $KT > $O/timeline.txt || exit 1
rm -rf $O/t
head -3 $O/timeline.txt
