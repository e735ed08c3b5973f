#!/bin/bash
# Quick GPU check: parity tests, then the bench (A/B over an env toggle when given).
# Usage (GPU box, repo root): bash tools/gpu_quick.sh TAG [ENV=VAL ...]
set -o pipefail
TAG=${1:-quick}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest_gpu exit $rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then tail -40 $OUT/pytest_gpu.log; exit $rc; fi
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'))"
for kv in "$@"; do
  env $kv timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $OUT/bench_$kv.json 2> $OUT/bench_$kv.err || { echo "bench $kv failed $?"; tail -20 $OUT/bench_$kv.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$kv.json')); print('bench $kv', d['value'], d['ms_per_step'])"
done
