# forward A/B of the attention variants, interleaved rounds on one box
set -o pipefail
for r in 1 2 3; do for v in 2 4; do
  VTD_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/fab_$v.log 2>&1 || { tail -5 gpurun_out/fab_$v.log; exit 1; }
  echo "v$v $(tail -1 gpurun_out/fab_$v.log | grep -o '"value": [0-9.]*') $(grep -o '"attention": {[^}]*}' gpurun_out/fab_$v.log | grep -o '"avg_us": [0-9.]*')"
done; done
