#!/bin/bash
# round 5: dynamic instruction mix (SALU / VALU / LDS / VMEM per MFMA) of every conv kernel family over one replay of
# every layer of the s@640 bs64 plan (tools/layer_bench.py), to rank the control-path overheads
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r05_insts; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU \
    SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- \
    python3 tools/layer_bench.py --reps 1 > $OUT/lb.log 2>&1 || exit 1
