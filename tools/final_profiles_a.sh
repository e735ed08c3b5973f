#!/bin/bash
# Round profile set, part A: full bench (with cpu_baseline), rocprofv3 kernel-trace + stats of the bench,
# per-stream step timeline, per-layer conv and BN timings.  Outputs under gpurun_out/$1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-finA}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "rocprof failed $?"; exit 1; }
KT=$(find $OUT/prof -name "*kernel_trace.csv" | head -1); KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
NF=$(python3 -c "import csv,sys; print(sum(int(r['Calls']) for r in csv.DictReader(open('$KS')) if 'prep_weights' in r['Name']))")
echo "forwards traced: $NF"
python3 $R/tools/prof_summary.py $KS $NF > $OUT/summary.txt && head -12 $OUT/summary.txt
python3 $R/tools/trace_streams.py $KT > $OUT/step_timeline.txt && head -8 $OUT/step_timeline.txt
timeout -k 10 300 python3 $R/tools/layer_bench.py > $OUT/layer_bench.txt 2> $OUT/layer.err || { echo "layer bench failed"; exit 1; }
tail -1 $OUT/layer_bench.txt
timeout -k 10 300 python3 $R/tools/bn_bench.py > $OUT/bn_bench.txt 2> $OUT/bn.err || { echo "bn bench failed"; exit 1; }
tail -1 $OUT/bn_bench.txt
