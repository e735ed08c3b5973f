#!/bin/bash
# round 5: fp16 packing (v_med3 + v_cvt_pk_f16_f32), one conversion per epilogue instance, conv_halo's hoisted geometry
# and soffset DMAs, conv_gemm's float-reciprocal pixel decompositions — parity, then same-box per-layer A/B against the
# library before these changes (ab/libyolomi_base.so = commit fcbffaf), then a bench line
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r05_epi; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_conv.py tests/test_gpu_bn.py -k "not in_model" > $OUT/test_conv.log 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_layers.py > $OUT/test_layers.log 2>&1 || exit 2
timeout -k 10 600 bash tools/lib_ab_layers.sh r05_epi/ab ab/libyolomi_base.so yolo-scratch_amd/libyolomi.so > $OUT/ab.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 4
