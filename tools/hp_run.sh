set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -x -q -k "hpipe" --timeout 120 --timeout-method thread > gpurun_out/r03e/hpipe_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r03e/hpipe_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/layer_bench.py --reps 10 > gpurun_out/r03e/layer_hpipe.txt 2> gpurun_out/r03e/layer.err || { tail -5 gpurun_out/r03e/layer.err; exit 1; }
timeout -k 10 300 python3 tools/layer_bench.py --reps 10 --hpipe 0 > gpurun_out/r03e/layer_nohpipe.txt 2> gpurun_out/r03e/layer0.err || exit 1
tail -1 gpurun_out/r03e/layer_hpipe.txt; tail -1 gpurun_out/r03e/layer_nohpipe.txt
