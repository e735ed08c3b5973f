#!/bin/bash
# Ablations of the pipelined conv (YM_PIPE_ABL=1: no MFMA, 2: no DMA) on pipe_check shapes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for abl in ${ABLS:-0 1 2}; do
  echo "== ABL $abl"
  YM_PIPE_ABL=$abl timeout -k 10 120 python3 $R/tools/pipe_check.py "$@" 2>&1 | grep -v amdgpu.ids | grep -v "ALL OK\|MISMATCHES"
done
