#!/bin/bash
# round 5: inference bench A/B over library policy settings (YM_LIB_SET strings, one per line in $1; "-" = defaults),
# s@640 bs 1 / 8, two interleaved repetitions on one box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_abset
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
mapfile -t CFGS < "$1"
for rep in 1 2; do
for i in "${!CFGS[@]}"; do
  c="${CFGS[$i]}"; [ "$c" = "-" ] && c=""
  YM_LIB_SET="$c" timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 --reps 100 --no-cpu-baseline > $O/c${i}_r$rep.json 2> $O/c${i}_r$rep.err || exit 1
  echo "rep $rep [${CFGS[$i]}] $(python -c "
import json
for l in open('$O/c${i}_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
