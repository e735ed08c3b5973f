#!/bin/bash
# s@128 gradient-error diagnostic under several kernel-path toggles (tools/diag_net.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/netdiag; mkdir -p $OUT
export TMPDIR=/tmp
for kv in "$@"; do
  echo "== $kv"
  env $kv timeout -k 10 200 python3 -u $R/tools/diag_net.py > $OUT/$kv.log 2>&1 || { echo "failed $?"; tail -5 $OUT/$kv.log; exit 1; }
  tail -4 $OUT/$kv.log
done
