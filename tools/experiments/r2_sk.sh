# stream-K pp2: parity, per-shape timing (SK off / on), forward bench (SK off / on)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 120 --timeout-method thread -k "stream_k or 256_tile or residual_in_place or statout" > gpurun_out/sk_tests.log 2>&1 || { tail -30 gpurun_out/sk_tests.log; exit 1; }
tail -2 gpurun_out/sk_tests.log
for m in 0 1; do
  VTD_GEMM_SK=$m timeout -k 10 200 python3 tools/gemm_bench.py --shapes qkv,attn_out,mlp1,mlp2,mlp3,head2 > gpurun_out/sk_gemm_$m.jsonl 2>&1 || { tail -5 gpurun_out/sk_gemm_$m.jsonl; exit 1; }
done
for m in 0 1 0 1; do
  VTD_GEMM_SK=$m timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sk_bench_$m.json 2>&1 || { tail -5 gpurun_out/sk_bench_$m.json; exit 1; }
  tail -1 gpurun_out/sk_bench_$m.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SK=$m', d['value'], d.get('roofline',{}).get('frac'))"
done
