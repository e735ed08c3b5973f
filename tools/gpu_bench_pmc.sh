#!/bin/bash
# The bench's two HBM counter passes (FETCH_SIZE, WRITE_SIZE: one counter per pass, kernel trace only) ->
# profiles/traffic.json families + probe (tools/pmc_traffic.py).  Outputs under gpurun_out/$1; $2 = source label.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-bpmc}; mkdir -p $OUT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/bpmc_$C -o run -- \
      python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bpmc_$C.err || { echo "bench pmc $C failed"; tail -5 $OUT/bpmc_$C.err; exit 1; }
done
BF=$(find $OUT/bpmc_FETCH_SIZE -name "*counter_collection.csv" | head -1); BW=$(find $OUT/bpmc_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_traffic.py $BF $BW $OUT/bench_FETCH_SIZE.json "${2:-profiles}" > $OUT/pmc_traffic.txt || { echo "pmc_traffic failed"; tail -5 $OUT/pmc_traffic.txt; exit 1; }
cat $OUT/pmc_traffic.txt
cp $R/profiles/traffic.json $OUT/traffic.json
rm -rf $OUT/bpmc_*
