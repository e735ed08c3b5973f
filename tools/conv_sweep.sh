#!/bin/bash
# A/B of conv kernel configurations on representative layers (tools/layer_bench.py), one process per config.
# Usage (GPU box, repo root): bash tools/conv_sweep.sh TAG "ENV=VAL ..." ...
set -o pipefail
TAG=${1:-sweep}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ONLY=${ONLY:-"1 3 6 8 11 24 48 71 73 78"}
i=0
for cfg in "base" "$@"; do
  if [ "$cfg" = base ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 200 python3 $R/tools/layer_bench.py --only $ONLY > $OUT/cfg$i.txt 2>&1 || { echo "cfg $cfg failed"; tail -5 $OUT/cfg$i.txt; exit 1; }
  echo "== $cfg"; grep -v amdgpu.ids $OUT/cfg$i.txt
  i=$((i+1))
done
