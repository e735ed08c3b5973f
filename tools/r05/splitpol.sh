#!/bin/bash
# round 5: eval small-grid policy A/B at bs 1 / 8 (K-split stage threshold x halo -> GEMM tile threshold), same box,
# interleaved; configurations as YM_LIB_SET strings
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05_splitpol
rm -rf $O; mkdir -p $O
cd $GRAFT_REPO_ROOT
CFGS=("ym_conv_set_eval_split_nk=12" "ym_conv_set_eval_split_nk=24" "ym_conv_set_eval_split_nk=24 ym_conv_set_eval_gemm_tiles=64" "ym_conv_set_eval_split_nk=18 ym_conv_set_eval_gemm_tiles=64" "ym_conv_set_eval_split_nk=12 ym_conv_set_eval_gemm_tiles=64" "ym_conv_set_eval_split=0 ym_conv_set_eval_gemm_tiles=64")
for rep in 1 2; do
for i in "${!CFGS[@]}"; do
  YM_LIB_SET="${CFGS[$i]}" timeout -k 10 300 python -u tools/infer_bench.py --batches 1 8 --reps 100 --no-cpu-baseline > $O/c${i}_r$rep.json 2> $O/c${i}_r$rep.err || exit 1
  echo "rep $rep [${CFGS[$i]}] $(python -c "
import json
for l in open('$O/c${i}_r$rep.json'):
    d = json.loads(l); print('bs%d %.3f ms %.0f img/s' % (d['batch'], d['ms_per_batch'], d['value']), end='  ')")"
done; done
