#!/bin/bash
# round 6: wgrad3 tap lookahead (wgrad3_kernel LA, ym_wgrad_set_lookahead; measurement library): bit-identity LA 1 vs 0,
# the conv parity test under LA 1, a same-process weight-gradient layer A/B, an in-step A/B
set -o pipefail
O=gpurun_out/r06_wgla
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
export YOLOMI_LIB=$PWD/yolo-scratch_amd/libyolomi_exp.so
timeout -k 10 300 python -u tools/r06/wg_parity.py > $O/parity.txt 2>&1 || { tail -20 $O/parity.txt; exit 1; }
tail -1 $O/parity.txt
timeout -k 10 500 python -u tools/pipe_ab.py ym_wgrad_set_lookahead --kinds wgrad --only 1 2 3 4 6 8 11 21 24 48 53 61 71 73 74 78 81 84 --variants 0 1 --rounds 3 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
cat $O/ab.txt
timeout -k 10 500 python -u tools/step_policy_ab.py ym_wgrad_set_lookahead --variants 0 1 --rounds 4 > $O/step_ab.txt 2>&1 || { tail -20 $O/step_ab.txt; exit 3; }
cat $O/step_ab.txt
