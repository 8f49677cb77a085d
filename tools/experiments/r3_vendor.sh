#!/bin/bash
# round 3 (final kernels): per-shape GEMM TFLOP/s next to the vendor library (torch.matmul ->
# hipBLASLt, timing reference only), two passes
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 env VTD_GEMM_REF_LIB=1 python3 tools/gemm_bench.py --reps 20 >> gpurun_out/r3_gemm_vendor.jsonl 2>/dev/null || exit 1
done
cat gpurun_out/r3_gemm_vendor.jsonl
