#!/bin/bash
# Per-layer conv timings (tools/layer_bench.py) under each kernel-selection policy, for picking selection rules
# layer by layer.  Outputs under gpurun_out/$1.  Usage (GPU box): bash tools/policy_sweep.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-sweep}; mkdir -p $OUT
run() {  # name, layer_bench args
  timeout -k 10 240 python3 $R/tools/layer_bench.py --reps 6 --names "${@:2}" > $OUT/lb_$1.txt 2> $OUT/lb_$1.err || { echo "$1 failed"; tail -5 $OUT/lb_$1.err; exit 1; }
  echo "$1: $(tail -1 $OUT/lb_$1.txt)"
}
run default
run pipe0 --pipe 0
run pipe2 --pipe 2
run halo0 --halo 0
run halo1 --halo 1
run hpipe0 --hpipe 0
run hpipe2 --hpipe 2
run direct0 --direct 0
