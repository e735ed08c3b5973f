set -o pipefail
O=gpurun_out/ab1; mkdir -p $O
export TMPDIR=/tmp
YM_CONV_TILE=2564 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 0 2564 0 2564; do
  YM_CONV_TILE=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
YM_CONV_TILE=0 timeout -k 10 300 python3 tools/layer_bench.py > $O/lb_0.txt 2>&1 || exit 1
YM_CONV_TILE=2564 timeout -k 10 300 python3 tools/layer_bench.py > $O/lb_2564.txt 2>&1 || exit 1
