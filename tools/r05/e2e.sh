#!/bin/bash
# round 5: eval end-to-end check — postprocess / eval tests, then the inference bench (bs 1 / 8 / 128) twice, and the
# bs-1 host profile of the end-to-end batch
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_e2e
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_post.py tests/test_gpu_eval_conv.py tests/test_gpu_determinism.py tests/test_gpu_model.py tests/test_gpu_modules.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
  timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 128 --reps 100 --no-cpu-baseline > $O/r$rep.json 2> $O/r$rep.err || exit 1
  echo "rep $rep $(python -c "
import json
for l in open('$O/r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done
timeout -k 10 200 python tools/host_prof.py 200 e2e > $O/host_prof_e2e.txt 2>&1 || exit 1
head -12 $O/host_prof_e2e.txt | tail -9
