#!/bin/bash
# Short round-3 GPU check: conv kernel parity, then per-layer timings of the 20-wide weight gradients and
# the halo-pipelined 3x3 layers (hpipe on / off).  Outputs under gpurun_out/$1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-quick}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_conv.log 2>&1
rc=$?; tail -3 $OUT/pytest_conv.log; [ $rc -ne 0 ] && { tail -30 $OUT/pytest_conv.log; exit $rc; }
timeout -k 10 200 python3 $R/tools/layer_bench.py --reps 6 --only 21 24 25 61 64 33 71 73 74 > $OUT/lb_default.txt 2> $OUT/lb.err || { tail -5 $OUT/lb.err; exit 1; }
cat $OUT/lb_default.txt
timeout -k 10 200 python3 $R/tools/layer_bench.py --reps 6 --hpipe 0 --only 71 73 74 > $OUT/lb_hpipe0.txt 2>> $OUT/lb.err || { tail -5 $OUT/lb.err; exit 1; }
cat $OUT/lb_hpipe0.txt
