#!/bin/bash
# direct-kernel check: conv parity tests, then layer timings of the stem-stage layers (A/B over env)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dirchk}; shift; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python3 $R/tools/layer_bench.py --only 1 2 3 4 5 > $OUT/layers.txt 2> $OUT/layers.err || { tail -20 $OUT/layers.err; exit 1; }
cat $OUT/layers.txt
for kv in "$@"; do
  env $kv timeout -k 10 300 python3 $R/tools/layer_bench.py --only 1 2 3 4 5 > $OUT/layers_$kv.txt 2>> $OUT/layers.err || exit 1
  echo "== $kv"; cat $OUT/layers_$kv.txt
done
