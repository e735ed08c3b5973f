#!/bin/bash
# round 5: training bench A/B over settings, one configuration per line in $1 ("-" = defaults): space-separated
# KEY=VAL items, ym_* keys are library setters (YM_LIB_SET), others environment variables; two interleaved
# repetitions on one box
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_benchset
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
mapfile -t CFGS < "$1"
for rep in ${REPS:-1 2}; do
for i in "${!CFGS[@]}"; do
  c="${CFGS[$i]}"; [ "$c" = "-" ] && c=""
  lib=""; envs=()
  for kv in $c; do case "$kv" in ym_*) lib="$lib $kv";; *) envs+=("$kv");; esac; done
  env "${envs[@]}" YM_LIB_SET="$lib" timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c${i}_r$rep.json 2> $O/c${i}_r$rep.err || { tail -5 $O/c${i}_r$rep.err; exit 1; }
  echo "rep $rep [${CFGS[$i]}] $(python -c "
import json
d = json.loads(open('$O/c${i}_r$rep.json').read().strip().splitlines()[-1]); print(d['value'], 'img/s', d['ms_per_step'], 'ms')")"
done; done
