#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_network.py $R/tests/test_gpu_boundary.py $R/tests/test_gpu_model.py -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "rc $?"; grep -E "PASS|FAIL|Error|worst|assert" $OUT/pytest.log | head -60
