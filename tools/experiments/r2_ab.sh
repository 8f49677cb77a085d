# A/B after a kernel change: kernel tests for the touched path, isolated GEMM shapes, bench
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -x --timeout 200 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/r2_ab_tests.log 2>&1 || { tail -30 gpurun_out/r2_ab_tests.log; exit 1; }
tail -1 gpurun_out/r2_ab_tests.log
timeout -k 10 200 python3 tools/gemm_bench.py --reps 10 --shapes ${SHAPES:-qkv,attn_out,mlp1,mlp1_noact,mlp2,mlp3,head2} > gpurun_out/r2_ab_gemm.jsonl 2>/dev/null || exit 1
cat gpurun_out/r2_ab_gemm.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_ab_bench.log 2>&1 || { tail -20 gpurun_out/r2_ab_bench.log; exit 1; }
tail -1 gpurun_out/r2_ab_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d['mfma_util_attn_mlp'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
