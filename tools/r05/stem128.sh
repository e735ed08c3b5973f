#!/bin/bash
# round 5: the eval stem's kernel time at bs 1 and bs 128 (rocprofv3 kernel trace of the inference bench)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_stem
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for B in 1 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t$B -o trace -- python3 $GRAFT_REPO_ROOT/tools/infer_bench.py --batches $B --reps 10 --no-cpu-baseline > $O/t$B.log 2>&1 || exit 1
  python3 $GRAFT_REPO_ROOT/tools/rocpd_summary.py $(find $O/t$B -name "*.db" | head -1) --top 40 > $O/t$B.txt || exit 1
  rm -rf $O/t$B
  echo "bs$B $(grep conv_first_eval $O/t$B.txt | cut -c1-60)"
done
