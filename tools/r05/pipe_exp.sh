#!/bin/bash
# round 5: per-wave tile size in the pipelined implicit GEMM — same-process A/B of the shipped 16-wave 256 x 128
# tile (32 x 64 per wave) against 8 waves of 64 x 64 (ym_pipe_set_exp 1), and SQ counter passes (LDS activity,
# MFMA busy, wave states) over ops 73 / 6 for both.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r05_pipe_exp; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pipe_ab.py ym_pipe_set_exp --only 6 10 11 20 47 48 52 73 74 78 79 \
    --variants 0 1 --reps 6 --rounds 3 > $OUT/ab.txt 2>&1 || exit 1
for v in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_v$v -o run -- \
      python3 tools/layer_bench.py --only 6 73 --reps 3 --set ym_pipe_set_exp=$v > $OUT/pmc_v$v.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
      --output-format csv -d $OUT/pmc2_v$v -o run -- \
      python3 tools/layer_bench.py --only 6 73 --reps 3 --set ym_pipe_set_exp=$v > $OUT/pmc2_v$v.log 2>&1 || exit 3
done
