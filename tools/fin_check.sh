#!/bin/bash
# BN finalize A/B (tools/fin_bench.py) after the BN / model parity tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-finchk}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_model.py $R/tests/test_gpu_bnfold.py $R/tests/test_gpu_determinism.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 200 python3 $R/tools/fin_bench.py > $OUT/fin.txt 2> $OUT/fin.err || { tail -20 $OUT/fin.err; exit 1; }
YM_BN_FIN1=0 timeout -k 10 200 python3 $R/tools/fin_bench.py > $OUT/fin_old.txt 2>> $OUT/fin.err || exit 1
cat $OUT/fin.txt; echo "== YM_BN_FIN1=0"; cat $OUT/fin_old.txt
