#!/bin/bash
# round 6: stride-2 data gradients — the 2-stage implicit GEMM (default) vs the pipelined kernel's generic 4-class path
# (ym_conv_set_pipe 2), same process
set -o pipefail
O=gpurun_out/r06_s2dgrad
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pipe_ab.py ym_conv_set_pipe --only 6 11 21 56 61 --variants -1 2 --kinds dgrad --rounds 3 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
grep "^op" $O/ab.txt
