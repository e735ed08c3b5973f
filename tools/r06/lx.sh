#!/bin/bash
# round 6: whole-network l / x steps vs the oracle at 256x256, and the remaining suite after the l test
set -o pipefail
O=gpurun_out/r06_lx
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_network.py -k "l_x" -m gpu -v -s --timeout 800 --timeout-method thread --durations=5 > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|worst|largest|^E " $O/pytest.log | head -30; tail -3 $O/pytest.log
exit $rc
