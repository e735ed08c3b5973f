#!/bin/bash
# Two-rank data-parallel rehearsal on a one-GPU box: bench.py and a short train_yolo11_cuda --synthetic
# run under torchrun with both ranks on GPU 0 and gloo all-reduces (RCCL needs one GPU per rank).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dp2}; mkdir -p $OUT
export TMPDIR=/tmp YM_DIST_BACKEND=gloo YM_DIST_DEVICE=0
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 $R/bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "dp bench failed $?"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
