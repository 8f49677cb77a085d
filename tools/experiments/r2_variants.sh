# A/B of the GEMM variants on the isolated forward shapes, one process per variant
set -o pipefail
for v in 10 7 11 5; do
  timeout -k 10 200 env VTD_GEMM_VARIANT=$v python3 tools/gemm_bench.py --reps 10 --shapes qkv,attn_out,mlp1,mlp1_noact,mlp2,mlp3,head2,sq8192 >> gpurun_out/r2_variants.jsonl 2>/dev/null || exit 1
done
echo ok
