#!/bin/bash
# Ping-pong conv kernels: parity tests, then same-process A/Bs against the current kernels on real layers.
# Usage (GPU box, repo root): bash tools/pp_check.sh TAG
set -o pipefail
TAG=${1:-pp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_conv.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pipe" > $OUT/pytest_pp.log 2>&1
rc=$?
echo "pytest exit $rc"; grep -E "passed|failed|Error" $OUT/pytest_pp.log | tail -5
[ $rc -ne 0 ] && { tail -40 $OUT/pytest_pp.log; exit $rc; }
timeout -k 10 300 python3 -u $R/tools/pipe_ab.py ym_conv_set_hpipe_pp --only 73 74 --variants 0 1 > $OUT/ab_hpp.txt 2> $OUT/ab_hpp.err
rc=$?
cat $OUT/ab_hpp.txt; [ $rc -ne 0 ] && { tail -20 $OUT/ab_hpp.err; exit $rc; }
timeout -k 10 300 python3 -u $R/tools/pipe_ab.py ym_conv_set_pipe_pp --only 10 48 52 78 --variants 0 1 > $OUT/ab_pp.txt 2> $OUT/ab_pp.err
rc=$?
cat $OUT/ab_pp.txt; [ $rc -ne 0 ] && { tail -20 $OUT/ab_pp.err; exit $rc; }
exit 0
