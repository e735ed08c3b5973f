#!/bin/bash
# Round profile set, part B: the two HBM counter passes of the bench (FETCH_SIZE, WRITE_SIZE; kernel
# trace only), then the inference and evaluation benches.  Outputs under gpurun_out/$1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-finB}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_fetch.json 2> $OUT/fetch.err || { echo "fetch pass failed $?"; tail -5 $OUT/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_write.json 2> $OUT/write.err || { echo "write pass failed $?"; tail -5 $OUT/write.err; exit 1; }
find $OUT -name "*counter_collection*"
timeout -k 10 300 python3 $R/tools/infer_bench.py --batches 1 8 128 > $OUT/infer_bench.json 2> $OUT/infer.err || { echo "infer failed"; tail -5 $OUT/infer.err; exit 1; }
cat $OUT/infer_bench.json | cut -c1-200
timeout -k 10 300 python3 $R/tools/eval_bench.py > $OUT/eval_bench.json 2> $OUT/eval.err || { echo "eval failed"; tail -5 $OUT/eval.err; exit 1; }
cat $OUT/eval_bench.json | cut -c1-300
