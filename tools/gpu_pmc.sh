#!/bin/bash
# HBM-traffic counters for the bench probe: two separate rocprofv3 --pmc passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass), kernel trace only, no runtime/sys tracing.
# Usage (GPU box, repo root): bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_fetch.json 2> $OUT/fetch.err || { echo "fetch pass failed $?"; tail -5 $OUT/fetch.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_write.json 2> $OUT/write.err || { echo "write pass failed $?"; tail -5 $OUT/write.err; exit 1; }
find $OUT -name "*counter_collection*"
