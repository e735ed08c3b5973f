#!/bin/bash
# round 5: weight-gradient control path — parity, then same-box per-layer A/B vs the library before the change
set -o pipefail
O=gpurun_out/r05_wg
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_layers.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
bash tools/lib_ab_layers.sh r05_wg/ab ab/libyolomi_base.so yolo-scratch_amd/libyolomi.so > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
grep -E "wgrad|total" $O/ab.txt | tail -45
