#!/bin/bash
# round 5, first GPU check: the ADVICE fixes (DP grad-write events, graph-safe accumulation, per-step pooled flag),
# the new BatchNorm tests (m*c >= 2^26 reduce + finalize vs fp64; fold vs two launches on in-model inputs) and the
# headline-geometry network test (s@640 bs64 vs the CPU oracle), then a default bench line.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05a
T="python -u -m pytest -v -s --timeout 120 --timeout-method thread"
timeout -k 10 200 $T tests/test_gpu_bn.py -k in_model > gpurun_out/r05a/fold.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 $T -x tests/test_gpu_bn.py tests/test_gpu_dp_world2.py tests/test_gpu_train_entry.py \
    tests/test_gpu_determinism.py tests/test_gpu_dp.py -k "not in_model" > gpurun_out/r05a/tests.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err || exit 3
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 680 --timeout-method thread tests/test_gpu_network.py \
    -k bs64 > gpurun_out/r05a/bs64.log 2>&1 || exit 4
