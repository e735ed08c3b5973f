#!/bin/bash
# Same-box A/B of two library builds (YOLOMI_LIB) on the BatchNorm streaming kernels (tools/bn_bench.py)
# and the bench step, interleaved A B A B.  Usage: bash tools/ab_bn.sh TAG LIB_A LIB_B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; A=$2; B=$3
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
for round in 1 2; do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    YOLOMI_LIB=$R/$L timeout -k 10 200 python3 $R/tools/bn_bench.py --reps 6 > $OUT/bn_${v}$round.txt 2>> $OUT/bn.err || { echo "bn bench $v failed"; tail -5 $OUT/bn.err; exit 1; }
    echo "$v$round $(tail -1 $OUT/bn_${v}$round.txt)"
    YOLOMI_LIB=$R/$L timeout -k 10 300 python3 $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}$round.json 2> $OUT/bench_${v}$round.err || { echo "bench $v failed"; tail -5 $OUT/bench_${v}$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}$round.json')); f=d['roofline_families']; print('$v$round', d['value'], d['ms_per_step'], 'bn', f['bn']['ms_per_step'], f['bn']['frac'])"
  done
done
