#!/bin/bash
# round 5: weight preparation A/B (ab/libyolomi_base.so = previous library vs the tree's), forward-only (eval) and
# forward + transposed (training) tables of s@640, interleaved, plus its bit-exact test
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_prep.py 2>&1 | tail -1 || exit 1
for rep in 1 2; do for lib in ${LIBS:-ab/libyolomi_base.so yolo-scratch_amd/libyolomi.so}; do for tr in "" "--train"; do
  r=$(YOLOMI_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python tools/prep_bench.py $tr) || exit 1; echo "rep $rep $lib $r"
done; done; done
