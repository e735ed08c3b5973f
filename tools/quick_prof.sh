#!/bin/bash
# Kernel-trace of tools/layer_bench.py on a few ops: per-kernel durations (rocprofv3 --stats).
# Usage: bash tools/quick_prof.sh TAG OP [OP ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/tools/layer_bench.py --reps 6 --only "$@" > $OUT/lb.txt 2> $OUT/lb.err || { tail -5 $OUT/lb.err; exit 1; }
cat $OUT/lb.txt
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$KS" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.2f} us  {float(r["TotalDurationNs"])/1e6:8.3f} ms  {r["Name"][:110]}')
PY
