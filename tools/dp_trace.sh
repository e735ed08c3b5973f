#!/bin/bash
# rocprofv3 kernel + memory-copy trace of the 2-rank data-parallel rehearsal on one GPU (gloo; RCCL refuses two
# ranks on one device): bench.py --gpus 2 starts the ranks itself.  Outputs under gpurun_out/$1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dptrace}; mkdir -p $OUT
export TMPDIR=/tmp
YM_DP_MARK=1 YM_DIST_BACKEND=gloo YM_DIST_DEVICE=0 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
    -d $OUT/prof -o run_%pid% -- python3 $R/bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench2.json 2> $OUT/bench2.err \
    || { echo "traced rehearsal failed $?"; tail -20 $OUT/bench2.err; exit 1; }
python3 $R/tools/dp_trace.py $OUT/prof > $OUT/dp_trace.txt && cat $OUT/dp_trace.txt
