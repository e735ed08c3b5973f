#!/bin/bash
# round 5: inference bench, previous library (ab/libyolomi_base.so) vs the tree's, bs $BATCHES, two interleaved
# repetitions on one box (YOLOMI_LIB picks the library)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_libab
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for lib in ab/libyolomi_base.so yolo-scratch_amd/libyolomi.so; do
  n=$(basename $lib .so)
  YOLOMI_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python -u tools/infer_bench.py --batches ${BATCHES:-1 8 128} --reps 100 --no-cpu-baseline > $O/${n}_r$rep.json 2> $O/${n}_r$rep.err || exit 1
  echo "rep $rep $n $(python -c "
import json
for l in open('$O/${n}_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s post %.1f us/img' % (d['batch'], d['ms_per_batch'], d['value'], d['postprocess']['us_per_image_gpu']), end='  ')")"
done; done
