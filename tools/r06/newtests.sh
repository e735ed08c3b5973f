#!/bin/bash
# round 6: the new parity tests + a baseline bench line on this box
set -o pipefail
O=gpurun_out/r06_newtests
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests/test_gpu_c5_eval.py tests/test_gpu_network.py::test_model_80_classes_train_step_vs_oracle "tests/test_gpu_network.py::test_model_l_x_train_step_vs_oracle" tests/test_gpu_train_entry.py::test_validate_through_pinned_worker_loader_with_eval_graph tests/test_gpu_network.py::test_model_ch3_train_step_vs_oracle tests/test_gpu_eval_conv.py tests/test_gpu_loss_nc.py tests/test_gpu_model.py -m gpu -v -s --timeout 1000 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|worst|level|kept|assert|passed|failed" $O/pytest.log | head -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
