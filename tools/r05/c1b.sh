#!/bin/bash
# round 5: parity of the new conv control paths (kernel tests, per-layer teacher-forced test at the bench's kernel
# selection) and a bench line
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r05_c1b; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_conv.py > $OUT/test_conv.log 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_layers.py > $OUT/test_layers.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 3
