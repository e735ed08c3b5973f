set -o pipefail
mkdir -p gpurun_out/pin
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pin/conv_tests.log 2>&1 || { tail -40 gpurun_out/pin/conv_tests.log; exit 1; }
tail -1 gpurun_out/pin/conv_tests.log
for V in "X=0" "YM_CONV_HALO=0"; do
  env $V timeout -k 10 240 python3 tools/layer_bench.py --reps 10 > gpurun_out/pin/$V.txt 2>&1 || exit 1
done
tail -1 gpurun_out/pin/*.txt
