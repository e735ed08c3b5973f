#!/bin/bash
# round 6: the whole-network tests (check_network's loss / items bound over the rounding model's draws)
set -o pipefail
O=gpurun_out/r06_net; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_network.py tests/test_gpu_model.py -m gpu -v -s --timeout 800 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|largest|^E " $O/pytest.log | head -40; tail -2 $O/pytest.log; exit $rc
