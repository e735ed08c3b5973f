#!/bin/bash
# Same-box A/B of one environment switch on the bench step, interleaved A B A B A B.
# Usage: bash tools/ab_env.sh TAG VAR VALUE_A VALUE_B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VAR=$2; A=$3; B=$4
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
for round in 1 2 3; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python3 $R/bench.py --steps 60 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}_$round.json 2> $OUT/bench_${v}_$round.err || { echo "bench $VAR=$v failed"; tail -5 $OUT/bench_${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$round.json')); print('$VAR=$v run $round', d['value'], d['ms_per_step'], 'c3', d['roofline']['frac'])"
  done
done
