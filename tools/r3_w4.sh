#!/bin/bash
# round 3: w4 GEMM correctness (GEMM kernel tests) + per-shape timing vs pp2 and the vendor library
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "gemm" > gpurun_out/r3_w4_tests.log 2>&1 || { tail -30 gpurun_out/r3_w4_tests.log; exit 1; }
tail -3 gpurun_out/r3_w4_tests.log
for v in 12 10; do
  VTD_GEMM_VARIANT=$v VTD_GEMM_REF_LIB=$([ $v = 12 ] && echo 1) timeout -k 10 200 python -u tools/gemm_bench.py --reps 20 --shapes qkv,attn_out,mlp1,mlp2,mlp3,head1,head2,sq8192 >> gpurun_out/r3_w4_bench.jsonl 2>&1 || exit 1
done
cat gpurun_out/r3_w4_bench.jsonl
