#!/bin/bash
# One GPU session: parity tests, the benchmark, and a rocprofv3 kernel-trace profile of it.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -m pytest $R/tests -m gpu -q > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest_gpu exit $rc"; tail -3 $OUT/pytest_gpu.log
# 0 = pass, 1 = test failures; anything else (fault, abort, timeout) ends the GPU session here
if [ $rc -gt 1 ]; then tail -30 $OUT/pytest_gpu.log; exit $rc; fi
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed $?"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 500 python3 $R/bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err
echo "rocprof exit $?"
find $OUT/prof -name "*stats*" | head
timeout -k 10 300 python3 $R/tools/eval_bench.py > $OUT/eval_bench.json 2> $OUT/eval_bench.err || { echo "eval bench failed $?"; tail -20 $OUT/eval_bench.err; exit 1; }
cat $OUT/eval_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_eval -o run -- \
    python3 $R/tools/eval_bench.py --reps 5 --cpu-images 5 > $OUT/prof_eval.json 2> $OUT/prof_eval.err
echo "rocprof eval exit $?"
