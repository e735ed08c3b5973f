#!/bin/bash
# Same-box A/B of two library builds (YOLOMI_LIB): the bench step and layer timings, interleaved A B A B.
# Usage: bash tools/ab_bench.sh TAG LIB_A LIB_B [layer ops...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; A=$2; B=$3; shift 3
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
for round in 1 2; do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    YOLOMI_LIB=$R/$L timeout -k 10 300 python3 $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}$round.json 2> $OUT/bench_${v}$round.err || { echo "bench $v failed"; tail -5 $OUT/bench_${v}$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}$round.json')); f=d['roofline_families']; print('$v$round', d['value'], d['ms_per_step'], 'c3', d['roofline']['frac'], 'fwd', f['fwd']['ms_per_step'], 'dgrad', f['dgrad']['ms_per_step'], 'wgrad', f['wgrad']['ms_per_step'])"
    if [ $# -gt 0 ]; then
      YOLOMI_LIB=$R/$L timeout -k 10 200 python3 $R/tools/layer_bench.py --reps 6 --only "$@" > $OUT/lb_${v}$round.txt 2>> $OUT/lb.err || { echo "layer bench $v failed"; exit 1; }
      tail -1 $OUT/lb_${v}$round.txt
    fi
  done
done
