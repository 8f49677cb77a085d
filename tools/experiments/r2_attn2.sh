set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r2_attn_tests.log 2>&1 || { tail -30 gpurun_out/r2_attn_tests.log; exit 1; }
tail -1 gpurun_out/r2_attn_tests.log
for v in 3 2; do
  VTD_ATTN_VARIANT=$v timeout -k 10 120 python3 tools/attn_bench.py >> gpurun_out/r2_attn_micro.jsonl 2>/dev/null || exit 1
done
cat gpurun_out/r2_attn_micro.jsonl
for v in 3 2; do
  VTD_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_attn_bench_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_attn_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH attn$v', d['value'], d['mfma_util_attn_mlp'], d['kernels']['attention']['avg_us'], d['roofline']['frac'])"
done
