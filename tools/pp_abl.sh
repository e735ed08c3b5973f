#!/bin/bash
# Ping-pong conv kernel ablations (timing only; ablated variants compute garbage): 1 normal, 2 no DMA in the
# loop, 3 no fragment reads in the loop; 0 = the 16-wave kernel
set -o pipefail
TAG=${1:-ppabl}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u $R/tools/pipe_ab.py ym_conv_set_pipe_pp --only 73 48 --variants 0 1 2 3 --also ym_conv_set_hpipe=0 > $OUT/ab.txt 2> $OUT/ab.err
rc=$?
cat $OUT/ab.txt; [ $rc -ne 0 ] && { tail -20 $OUT/ab.err; exit $rc; }
exit 0
