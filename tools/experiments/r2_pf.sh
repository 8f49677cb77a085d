# L2-prefetch variants of pp2 (VTD_GEMM_VARIANT 40 = PFD 3, 41 = PFD 4): GEMM tests under
# variant 40, then isolated shapes for 10 / 40 / 41 interleaved, then the forward bench
set -o pipefail
VTD_GEMM_VARIANT=40 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k gemm --timeout 120 --timeout-method thread > gpurun_out/r2_pf_tests.log 2>&1 || { tail -30 gpurun_out/r2_pf_tests.log; exit 1; }
tail -1 gpurun_out/r2_pf_tests.log
for v in 10 40 41 10 40 41; do
  timeout -k 10 200 env VTD_GEMM_VARIANT=$v python3 tools/gemm_bench.py --reps 10 --shapes ${SHAPES:-qkv,attn_out,mlp1,mlp2,mlp3,sq8192} >> gpurun_out/r2_pf.jsonl 2>/dev/null || exit 1
done
cat gpurun_out/r2_pf.jsonl
for v in 10 40 41; do
  VTD_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_pf_bench_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_pf_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $v', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'])"
done
