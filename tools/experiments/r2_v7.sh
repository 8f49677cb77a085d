set -o pipefail
for v in 10 7 11; do
  timeout -k 10 200 env VTD_GEMM_VARIANT=$v python3 tools/gemm_bench.py --reps 10 --shapes qkv,attn_out,mlp1,mlp2,mlp3 >> gpurun_out/r2_v7.jsonl 2>/dev/null || exit 1
done
cat gpurun_out/r2_v7.jsonl
for v in 10 7 11; do
  VTD_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_v7_bench_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_v7_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH v$v', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'])"
done
