#!/bin/bash
# Round-3 GPU session: parity tests, the driver's exact bench command, its rocprofv3 kernel-trace summary,
# and the per-layer counter passes behind the 3x3 family's traffic.  Outputs under gpurun_out/$1.
# Usage (GPU box, repo root): bash tools/gpu_r03.sh TAG [skip-tests|tests] [short]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 500 python3 -u -m pytest $R/tests -m gpu -x -q -s --timeout 120 --timeout-method thread $PYTEST_EXTRA > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_gpu exit $rc"; tail -3 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ]; then tail -40 $OUT/pytest_gpu.log; exit $rc; fi
fi
timeout -k 10 400 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "rocprof failed $?"; tail -5 $OUT/prof_bench.err; exit 1; }
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
NF=$(python3 -c "import csv; print(sum(int(r['Calls']) for r in csv.DictReader(open('$KS')) if 'prep_weights' in r['Name']))")
echo "forwards traced: $NF"
python3 $R/tools/prof_summary.py $KS $NF > $OUT/summary.txt && head -14 $OUT/summary.txt
timeout -k 10 300 python3 $R/tools/layer_bench.py --reps 4 > $OUT/layer_bench.txt 2> $OUT/layer.err || { echo "layer bench failed"; tail -5 $OUT/layer.err; exit 1; }
tail -1 $OUT/layer_bench.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- \
      python3 $R/tools/layer_bench.py --reps 2 --seq-out $OUT/seq.json > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$C.log; exit 1; }
done
F=$(find $OUT/pmc_FETCH_SIZE -name "*counter_collection.csv" | head -1)
W=$(find $OUT/pmc_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_layers.py $F $W $OUT/seq.json profiles/r03 > $OUT/pmc_layers.txt && tail -3 $OUT/pmc_layers.txt
cp $R/profiles/traffic.json $OUT/traffic.json
[ "$3" = "short" ] && exit 0
timeout -k 10 300 python3 $R/tools/miopen_ref.py > $OUT/miopen_ref.txt 2> $OUT/miopen_ref.err || { echo "miopen ref failed"; tail -5 $OUT/miopen_ref.err; }
cat $OUT/miopen_ref.txt
bash $R/tools/pmc_conv.sh $OUT/pmc73 73 && python3 $R/tools/pmc_summary.py $OUT/pmc73 > $OUT/pmc73_summary.txt; cat $OUT/pmc73_summary.txt
# last: the 3-stream HIP-graph capture (segfaulted in round 2) under faulthandler
YM_GRAPH=1 YM_STREAMS=3 timeout -k 10 180 python3 -X faulthandler $R/tools/graph_debug.py full > $OUT/graph3.log 2>&1
echo "graph3 exit $?"; tail -40 $OUT/graph3.log
