#!/bin/bash
# round 5: conv_pipe's single-class control path (C1) and conv_hpipe's counted (division-free) position state —
# parity (conv kernel tests + per-layer teacher-forced test), same-process A/B against the generic control path
# (ym_pipe_set_exp 20) and hpipe vs pipe on the 128-channel 3x3 layers (ym_conv_set_hpipe 2), instruction counts.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r05_c1; mkdir -p $OUT
rm -f $OUT/*.log $OUT/*.txt
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_conv.py > $OUT/test_conv.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/pipe_ab.py ym_pipe_set_exp --only 6 10 11 12 20 22 33 47 48 52 73 74 78 79 \
    --variants 0 20 --reps 6 --rounds 4 > $OUT/ab.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/pipe_ab.py ym_conv_set_hpipe --only 8 9 53 72 73 74 48 58 78 79 \
    --variants 1 2 --reps 6 --rounds 4 > $OUT/ab_hpipe.txt 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM --output-format csv -d $OUT/sq2 -o run -- \
    python3 tools/layer_bench.py --only 73 8 --reps 3 > $OUT/sq2.log 2>&1 || exit 4
timeout -k 10 900 $T tests/test_gpu_layers.py > $OUT/test_layers.log 2>&1 || exit 5
