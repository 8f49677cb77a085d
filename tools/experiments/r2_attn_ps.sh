# persistent short-sequence attention (VTD_ATTN_VARIANT 4) vs the per-pair kernel (2):
# attention kernel tests, C2 micro-benchmark interleaved, forward bench with each
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/ps_tests.log 2>&1 || { tail -30 gpurun_out/ps_tests.log; exit 1; }
tail -1 gpurun_out/ps_tests.log
for r in 1 2 3; do for v in 2 4; do
  VTD_ATTN_VARIANT=$v timeout -k 10 120 python3 tools/attn_bench.py >> gpurun_out/ps_micro.jsonl 2>/dev/null || exit 1
done; done
cat gpurun_out/ps_micro.jsonl
for v in 2 4; do
  VTD_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ps_bench_$v.log 2>&1 || { tail -5 gpurun_out/ps_bench_$v.log; exit 1; }
  tail -1 gpurun_out/ps_bench_$v.log | cut -c1-200
  grep -o '"attention": {[^}]*}' gpurun_out/ps_bench_$v.log
done
