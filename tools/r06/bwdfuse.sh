#!/bin/bash
# round 6: the one-launch BatchNorm backward on the small maps (ym_bn_bwd_fused) — parity, then an in-step A/B
# (YM_BWD_FUSE=1 shipped vs 0: ym_bn_bwd_reduce_fold + ym_bn_bwd_apply[_res]), interleaved pairs on one box
set -o pipefail
O=gpurun_out/r06_bwdfuse
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_determinism.py "tests/test_gpu_model.py::test_model_n320_train_step_vs_reference" -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for f in 1 0; do
  YM_BWD_FUSE=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 100 > $O/bench_f${f}_r$rep.json 2> $O/bench_f${f}_r$rep.err || { tail -5 $O/bench_f${f}_r$rep.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$O/bench_f${f}_r$rep.json').read().strip().splitlines()[-1]);print('fuse=$f rep=$rep', d['value'], d['ms_per_step'], d['roofline_families']['bn'].get('ms'))"
done; done
