#!/bin/bash
# round 3 (final kernels): bench lines of the other BASELINE configs + the MX GEMM variant A/B at
# C5 fp8 (1 = ping-pong, 3 = x4 for K >= 2048)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/r03_bench_${n}_s5.log 2>&1 || { tail -5 gpurun_out/r03_bench_${n}_s5.log; return 1; }
  tail -1 gpurun_out/r03_bench_${n}_s5.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$n', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'], d['kernels']['attention']['avg_us'], d['kernels']['layernorm']['avg_us'])"
}
run c5_b128_fp8 --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 &&
run c5_b128_fp8b --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 &&
run c5_b128_bf16 --preset vit_l16_384 --batch 128 --steps 10 --warmup 3 &&
run c2_b64_bf16 --batch 64 --steps 20 --warmup 5 &&
run c3_b32_bf16 --preset vit_b16_640 --batch 32 --steps 10 --warmup 3 &&
run c2_b256_f32 --dtype f32 --batch 256 --steps 5 --warmup 2
