# attention A/B: kernel tests (default and VTD_ATTN_VARIANT=4), then the forward bench under
# variant 3 (the previous default at N > 128: chunked 8-wave kernel) and 2 (whole-pair kernel)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -x -k "attention or c2 or tiny or two_stream" --timeout 120 --timeout-method thread > gpurun_out/r2_attn_tests.log 2>&1 || { tail -30 gpurun_out/r2_attn_tests.log; exit 1; }
tail -1 gpurun_out/r2_attn_tests.log
VTD_ATTN_VARIANT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r2_attn_tests4.log 2>&1 || { tail -30 gpurun_out/r2_attn_tests4.log; exit 1; }
tail -1 gpurun_out/r2_attn_tests4.log
for v in 3 2 3 2; do
  VTD_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_attn_bench_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_attn_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH attn$v', d['value'], d['mfma_util_attn_mlp'], d['kernels']['attention']['avg_us'], d['roofline']['frac'])"
done
