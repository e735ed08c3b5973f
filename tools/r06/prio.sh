#!/bin/bash
# round 6: stream priorities — the scheduler's streams at high priority (YM_STREAM_PRIO=1) vs the shipped default,
# in-step A/B, interleaved pairs on one box; a determinism/parity check under the variant first
set -o pipefail
O=gpurun_out/r06_prio
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
YM_STREAM_PRIO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_determinism.py "tests/test_gpu_model.py::test_model_n320_train_step_vs_reference" tests/test_gpu_dp.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for f in 1 0; do
  YM_STREAM_PRIO=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 100 > $O/bench_p${f}_r$rep.json 2> $O/bench_p${f}_r$rep.err || { tail -5 $O/bench_p${f}_r$rep.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$O/bench_p${f}_r$rep.json').read().strip().splitlines()[-1]);print('prio=$f rep=$rep', d['value'], d['ms_per_step'])"
done; done
