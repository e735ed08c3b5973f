set -o pipefail
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/nms4
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_post.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nms_t.log 2>&1 || { tail -30 gpurun_out/nms_t.log; exit 1; }
tail -1 gpurun_out/nms_t.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nms4/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/infer_bench.py --no-cpu-baseline --reps 5 > $GRAFT_REPO_ROOT/gpurun_out/nms4/infer.json 2>&1; echo "rocprof $?"
cd /tmp && YM_NMS_BITMASK=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nms4/prof_off -o run -- python3 $GRAFT_REPO_ROOT/tools/infer_bench.py --no-cpu-baseline --reps 5 --batches 1 > /dev/null 2>&1; echo "rocprof $?"
