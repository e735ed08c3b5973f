#!/bin/bash
# Stall-analysis counter passes over one conv layer's three kernels (tools/layer_bench.py --only OP).
# Usage (GPU box, repo root): bash tools/pmc_conv.sh OUTDIR OP [extra layer_bench args, e.g. --hpipe 0]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; OP=${2:-6}; EXTRA="${@:3}"
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$tag -o run -- \
      python3 tools/layer_bench.py --only $OP --reps 3 $EXTRA > $OUT/$tag.log 2>&1 || { echo "pass $tag failed $?"; return 1; }
}
run p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA && \
run p2 SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE && \
run p3 TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE GRBM_COUNT
