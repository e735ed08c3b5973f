set -o pipefail
mkdir -p gpurun_out/abl
for A in none nomma nodma; do
  YM_CONV_ABLATE=$A timeout -k 10 200 python3 tools/layer_bench.py --only 6 11 48 73 21 5 52 --reps 20 > gpurun_out/abl/$A.txt 2>&1 || exit 1
done
YM_CONV_TILE=256 timeout -k 10 200 python3 tools/layer_bench.py --only 6 11 48 73 21 5 52 --reps 20 > gpurun_out/abl/t256.txt 2>&1 || exit 1
