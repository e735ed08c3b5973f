#!/bin/bash
# round 5: what bounds conv_pipe — same-process ablations (ym_pipe_set_exp 10: every stage DMA out of range, 11: no
# MFMAs, 12: only the input's DMAs out of range, 13: only the weights') and memory-path counters of op 73's forward.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r05_pipe_abl; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pipe_ab.py ym_pipe_set_exp --only 10 52 73 78 11 6 \
    --variants 0 10 11 12 13 --reps 6 --rounds 3 > $OUT/abl.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum \
    TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/mem -o run -- python3 tools/layer_bench.py --only 73 --reps 3 > $OUT/mem.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/sq -o run -- \
    python3 tools/layer_bench.py --only 73 --reps 3 > $OUT/sq.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM --output-format csv -d $OUT/sq2 -o run -- \
    python3 tools/layer_bench.py --only 73 --reps 3 > $OUT/sq2.log 2>&1 || exit 4
