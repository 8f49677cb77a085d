# C2 at B = 64: one stream vs two parts (VTD_SPLIT_MIN_TILES lowered) vs 4 parts
set -o pipefail
for cfg in "1 48" "2 16" "4 8" "1 48" "2 16"; do
  set -- $cfg
  VTD_SPLIT_MIN_TILES=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --batch 64 --streams $1 > gpurun_out/r2_b64_$1.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_b64_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH B64 streams=$1', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'], d['ms_per_step'])"
done
