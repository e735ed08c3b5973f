#!/bin/bash
# eval-path check: parity tests that run eval forwards, then the inference bench (bs1 / bs8 / bs128)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-evalchk}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_model.py $R/tests/test_gpu_boundary.py $R/tests/test_gpu_post.py $R/tests/test_gpu_train_entry.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python3 $R/tools/infer_bench.py --batches 1 8 128 --no-cpu-baseline > $OUT/infer.json 2> $OUT/infer.err || { tail -20 $OUT/infer.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/infer.json'):
    d=json.loads(l); print(d['batch'], d['value'], d['ms_per_batch'], d['postprocess']['us_per_image_gpu'], d['postprocess']['bit_exact_vs_oracle'])"
