#!/bin/bash
# round 6: (1) SQ counters of op 73 / op 6 under each conv_pipe MFMA shape (ym_conv_set_pipe_mfma 0 / 1 / 2: the
# 16x16x32 shipped kernel, 32x32x16 on the same 16-wave tile, 32x32x16 on 8 waves of 64 x 64); (2) the step's
# wall-time share per kernel family (tools/step_ablate.py)
set -o pipefail
O=gpurun_out/r06_diag1
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
# the MFMA-shape setter lives in the measurement library (make -C yolo-scratch_amd/csrc exp)
export YOLOMI_LIB=$PWD/yolo-scratch_amd/libyolomi_exp.so
for v in 0 1 2; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_v$v -o run -- \
      python3 tools/layer_bench.py --only 6 73 --reps 3 --set ym_conv_set_pipe_mfma=$v > $O/pmc_v$v.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
      SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2_v$v -o run -- \
      python3 tools/layer_bench.py --only 6 73 --reps 3 --set ym_conv_set_pipe_mfma=$v > $O/pmc2_v$v.log 2>&1 || exit 3
done
unset YOLOMI_LIB
echo counters done
timeout -k 10 400 python -u tools/step_ablate.py --steps 20 --rounds 3 > $O/ablate.txt 2>&1 || { tail -20 $O/ablate.txt; exit 4; }
cat $O/ablate.txt
