#!/bin/bash
# round 5: inference bench A/B over settings (one per line in $1, "-" = defaults; ym_* = library setters), bs $BATCHES
# (default 8 128), two interleaved repetitions on one box; with $TESTS set, the eval tests run first under each setting
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_abinf
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
mapfile -t CFGS < "$1"
if [ -n "$TESTS" ]; then for i in "${!CFGS[@]}"; do
  c="${CFGS[$i]}"; [ "$c" = "-" ] && c=""
  YM_LIB_SET="$c" timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $O/t$i.log 2>&1 || { grep -E "^(FAILED|E )" $O/t$i.log | head; exit 1; }
  echo "[${CFGS[$i]}] $(tail -1 $O/t$i.log)"
done; fi
for rep in 1 2; do
for i in "${!CFGS[@]}"; do
  c="${CFGS[$i]}"; [ "$c" = "-" ] && c=""
  YM_LIB_SET="$c" timeout -k 10 300 python -u tools/infer_bench.py --batches ${BATCHES:-8 128} --reps 100 --no-cpu-baseline > $O/c${i}_r$rep.json 2> $O/c${i}_r$rep.err || exit 1
  echo "rep $rep [${CFGS[$i]}] $(python -c "
import json
for l in open('$O/c${i}_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
