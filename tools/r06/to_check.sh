#!/bin/bash
# round 6: the tap-innermost rule shipped (stride-2 3x3 forwards on >= 128-wide maps): conv + teacher-forced layer
# parity with the shipping library, the in-step A/B (rule vs chunk-innermost everywhere) in the measurement library,
# and the bench line
set -o pipefail
O=gpurun_out/r06_to
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_layers.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
YOLOMI_LIB=$PWD/yolo-scratch_amd/libyolomi_exp.so timeout -k 10 500 python -u tools/step_policy_ab.py ym_conv_set_pipe_taporder --variants 0 -1 --rounds 5 > $O/step_ab.txt 2>&1 || { tail -20 $O/step_ab.txt; exit 2; }
grep -v amdgpu.ids $O/step_ab.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
python3 -c "
import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_probe']['frac'], d['roofline_probe']['kernel'][:60])"
