#!/bin/bash
# HIP-graph replay of the training step at 3 scheduler streams: capture check (faulthandler), the graph
# determinism tests, then the bench step eager vs graph (2 and 3 streams) in one call.  Outputs gpurun_out/$1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-graph}; mkdir -p $OUT
YM_GRAPH=1 YM_STREAMS=3 timeout -k 10 150 python3 -X faulthandler $R/tools/graph_debug.py full > $OUT/capture3.log 2>&1 || { echo "capture failed $?"; tail -30 $OUT/capture3.log; exit 1; }
tail -2 $OUT/capture3.log
timeout -k 10 200 python3 -u -m pytest $R/tests/test_gpu_determinism.py -x -q --timeout 120 --timeout-method thread > $OUT/det.log 2>&1 || { echo "determinism failed"; tail -30 $OUT/det.log; exit 1; }
tail -1 $OUT/det.log
run_bench() {   # $1 tag; YM_GRAPH / YM_STREAMS set by the caller
  timeout -k 10 300 python3 $R/bench.py --steps 60 --warmup 5 --no-cpu-baseline > $OUT/bench_$1.json 2> $OUT/bench_$1.err || { echo "bench $1 failed"; tail -5 $OUT/bench_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$1.json')); print('$1', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
}
YM_GRAPH=0 run_bench eager && YM_GRAPH=1 YM_STREAMS=3 run_bench graph3 && YM_GRAPH=1 YM_STREAMS=2 run_bench graph2 && YM_GRAPH=0 run_bench eager_b
