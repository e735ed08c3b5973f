#!/bin/bash
# Round-6 profile set at HEAD (outputs under gpurun_out/$1, then copied into profiles/r06/at_<commit> by hand):
#  1. the driver's bench command (with the CPU baseline);
#  2. rocprofv3 --kernel-trace --stats of exactly that command -> summary.txt, kernel_stats.csv, step timeline;
#  3. the per-launch -> layer map: one single-stream step under rocprofv3 --kernel-trace, joined with the
#     recorded library calls (tools/launch_map.py) -> layer_map.txt (the 3x3 family recomputed from the trace);
#  4. per-layer conv timings (kernel names) and BatchNorm timings;
#  5. HBM counter passes (FETCH_SIZE, WRITE_SIZE; one counter per pass) over the bench (families + probe) and
#     over the layer replay (per layer, 3x3 family) -> profiles/traffic.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prof06}; mkdir -p $OUT
SRC=${2:-profiles/r06}
export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "rocprof failed $?"; tail -5 $OUT/prof_bench.err; exit 1; }
KS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); KT=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
NF=$(python3 -c "import csv; print(sum(int(r['Calls']) for r in csv.DictReader(open('$KS')) if 'prep_weights' in r['Name']))")
echo "forwards traced: $NF"
python3 $R/tools/prof_summary.py $KS $NF > $OUT/summary.txt && head -8 $OUT/summary.txt
python3 $R/tools/trace_streams.py $KT > $OUT/step_timeline.txt && head -7 $OUT/step_timeline.txt
cp $KS $OUT/kernel_stats.csv
rm -f $KT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lmap -o run -- \
    python3 $R/tools/launch_map.py record $OUT/calls.json > $OUT/lmap.log 2>&1 || { echo "launch map record failed"; tail -5 $OUT/lmap.log; exit 1; }
LT=$(find $OUT/lmap -name "*kernel_trace.csv" | head -1)
python3 $R/tools/launch_map.py join $LT $OUT/calls.json > $OUT/layer_map.txt || { echo "join failed"; tail -5 $OUT/layer_map.txt; exit 1; }
tail -14 $OUT/layer_map.txt
timeout -k 10 300 python3 $R/tools/layer_bench.py --reps 6 --names > $OUT/layer_bench.txt 2> $OUT/layer.err || { echo "layer bench failed"; tail -5 $OUT/layer.err; exit 1; }
tail -1 $OUT/layer_bench.txt
timeout -k 10 300 python3 $R/tools/bn_bench.py > $OUT/bn_bench.txt 2> $OUT/bn.err || { echo "bn bench failed"; tail -5 $OUT/bn.err; exit 1; }
tail -1 $OUT/bn_bench.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/bpmc_$C -o run -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bpmc_$C.err || { echo "bench pmc $C failed"; tail -5 $OUT/bpmc_$C.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $OUT/lpmc_$C -o run -- \
      python3 $R/tools/layer_bench.py --reps 2 --seq-out $OUT/seq.json > $OUT/lpmc_$C.log 2>&1 || { echo "layer pmc $C failed"; tail -5 $OUT/lpmc_$C.log; exit 1; }
done
BF=$(find $OUT/bpmc_FETCH_SIZE -name "*counter_collection.csv" | head -1); BW=$(find $OUT/bpmc_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_traffic.py $BF $BW $OUT/bench_FETCH_SIZE.json "$SRC" > $OUT/pmc_traffic.txt && cat $OUT/pmc_traffic.txt
LF=$(find $OUT/lpmc_FETCH_SIZE -name "*counter_collection.csv" | head -1); LW=$(find $OUT/lpmc_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_layers.py $LF $LW $OUT/seq.json "$SRC" > $OUT/pmc_layers.txt && tail -3 $OUT/pmc_layers.txt
cp $R/profiles/traffic.json $OUT/traffic.json
rm -rf $OUT/bpmc_* $OUT/lpmc_*
