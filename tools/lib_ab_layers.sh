#!/bin/bash
# Same-box per-layer A/B of two library builds (YOLOMI_LIB), interleaved A B A B, then a per-(op, direction)
# comparison (tools/lib_ab_compare.py).  Usage (GPU box): bash tools/lib_ab_layers.sh TAG LIB_A LIB_B [ops...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; A=$2; B=$3; shift 3
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
ONLY=""; [ $# -gt 0 ] && ONLY="--only $*"
for round in 1 2; do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    YOLOMI_LIB=$R/$L timeout -k 10 240 python3 $R/tools/layer_bench.py --reps 8 --names $ONLY > $OUT/lb_${v}$round.txt 2>> $OUT/lb.err || { echo "layer bench $v failed"; tail -5 $OUT/lb.err; exit 1; }
  done
done
python3 $R/tools/lib_ab_compare.py $OUT
