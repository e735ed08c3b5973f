#!/bin/bash
# round 6: conv_pipe loop form (LP 0 flat / 1 nested, ym_conv_set_pipe_loop, measurement library) — parity on every
# forced-pipe shape, then a same-process layer A/B on the s@640 bs64 plan's pipelined layers, then counters of both
set -o pipefail
O=gpurun_out/r06_loop
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
export YOLOMI_LIB=$PWD/yolo-scratch_amd/libyolomi_exp.so
timeout -k 10 300 python -u tools/r06/loop_parity.py ym_conv_set_pipe_loop 1 > $O/parity1.txt 2>&1 && timeout -k 10 300 python -u tools/r06/loop_parity.py ym_conv_set_pipe_loop 2 > $O/parity.txt 2>&1 || { tail -20 $O/parity*.txt; exit 1; }
tail -1 $O/parity.txt
timeout -k 10 500 python -u tools/pipe_ab.py ym_conv_set_pipe_loop --only 6 10 11 52 73 74 78 48 47 71 8 53 --variants 0 1 2 --rounds 3 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
cat $O/ab.txt
timeout -k 10 500 python -u tools/step_policy_ab.py ym_conv_set_pipe_loop --variants 0 1 2 --rounds 4 > $O/step_ab.txt 2>&1 || { tail -20 $O/step_ab.txt; exit 3; }
cat $O/step_ab.txt
