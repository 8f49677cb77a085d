# Per-shape GEMM TFLOP/s of the current kernels next to the vendor library (torch.matmul ->
# hipBLASLt, timing reference only), same process, same random operands.
set -o pipefail
timeout -k 10 300 env VTD_GEMM_REF_LIB=1 python3 tools/gemm_bench.py --reps 20 ${SHAPES:+--shapes $SHAPES} > gpurun_out/r2_gemm_vendor.jsonl 2>/dev/null || exit 1
cat gpurun_out/r2_gemm_vendor.jsonl
