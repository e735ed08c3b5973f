#!/bin/bash
# Counter passes over the pipelined conv (tools/pipe_check.py SHAPE).  Usage: bash tools/pipe_pmc.sh OUT SHAPE
set -o pipefail
OUT=${1:-gpurun_out/ppmc}; SH=${2:-0}
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$tag -o run -- \
      python3 tools/pipe_check.py $SH > $OUT/$tag.log 2>&1 || { echo "pass $tag failed $?"; tail -3 $OUT/$tag.log; return 1; }
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA && \
run p2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE && \
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
for path in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"]
        if "conv_pipe" not in k and "conv_gemm" not in k and "halo" not in k:
            continue
        short = ("pipe" if "conv_pipe" in k else "gemm" if "conv_gemm" in k else "halo") + ("_d" if ("ELi1E" in k.split("PipeArgs")[0][-12:] or ", 1>" in k) else "")
        agg[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in agg.items():
        print(k)
        print("   " + "  ".join(f"{n}={sum(v)/len(v):.4g}" for n, v in sorted(c.items())))
PY
