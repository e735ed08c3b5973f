#!/bin/bash
# round 6: conv_pipe K order (conv_pipe_kernel TO 0 chunk-innermost / 1 tap-innermost; ym_conv_set_pipe_taporder,
# measurement library): parity on every forced-pipe shape, layer A/B, HBM fetch counters per layer, in-step A/B
set -o pipefail
O=gpurun_out/r06_taporder
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
export YOLOMI_LIB=$PWD/yolo-scratch_amd/libyolomi_exp.so
timeout -k 10 300 python -u tools/r06/loop_parity.py ym_conv_set_pipe_taporder 1 > $O/parity.txt 2>&1 || { tail -20 $O/parity.txt; exit 1; }
tail -1 $O/parity.txt
timeout -k 10 500 python -u tools/pipe_ab.py ym_conv_set_pipe_taporder --only 6 10 11 52 73 74 78 48 47 71 --variants 0 1 --rounds 3 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
grep -v amdgpu.ids $O/ab.txt
for v in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_v$v -o run -- \
      python3 tools/layer_bench.py --only 6 11 73 74 78 --reps 3 --set ym_conv_set_pipe_taporder=$v > $O/pmc_v$v.log 2>&1 || exit 3
  echo "== TO $v"; python3 tools/r06/pmc_kern.py $O/pmc_v$v conv_pipe
done
timeout -k 10 500 python -u tools/step_policy_ab.py ym_conv_set_pipe_taporder --variants 0 1 --rounds 4 > $O/step_ab.txt 2>&1 || { tail -20 $O/step_ab.txt; exit 4; }
grep -v amdgpu.ids $O/step_ab.txt
