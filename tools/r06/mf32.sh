#!/bin/bash
# round 6: 32x32x16 MFMA instances of conv_pipe — parity (forced pipe, every MFMA shape), then a same-process layer A/B
# (ym_conv_set_pipe_mfma 0 / 1 / 2) on the s@640 bs64 plan's pipelined layers, then the bench line at the default
set -o pipefail
O=gpurun_out/r06_mf32
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -k "pipe_kernel or hpipe_kernel" -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/pipe_ab.py ym_conv_set_pipe_mfma --setter2 ym_conv_set_pipe_order --only 6 10 11 52 73 74 78 48 47 71 8 53 --variants 0:0 0:1 1:0 2:0 2:1 --rounds 3 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
cat $O/ab.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
tail -c 400 $O/bench.json
