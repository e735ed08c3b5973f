#!/bin/bash
# Round-4 GPU check: the whole GPU suite, the kernel-policy sweep, and the C4 / C5 configurations
# (m@1280 bs16 training step; s@640 inference bs1 / bs8 / bs128 + postprocess).  Outputs under gpurun_out/$1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04}; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 800 python3 -u -m pytest $R/tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/pytest_gpu.log | tail -20; exit $rc; }
fi
bash $R/tools/policy_sweep.sh ${1:-r04}/sweep || exit 1
timeout -k 10 300 python3 $R/bench.py --scale m --imgsz 1280 --batch 16 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4_m1280.json 2> $OUT/c4.err || { tail -5 $OUT/c4.err; exit 1; }
echo "C4: $(tail -1 $OUT/c4.err)"
timeout -k 10 300 python3 $R/tools/infer_bench.py --batches 1 8 128 --no-cpu-baseline > $OUT/c5_infer.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
cat $OUT/c5_infer.json | cut -c1-300
