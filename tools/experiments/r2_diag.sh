# pp2 main-loop timing diagnostics (VTD_GEMM_VARIANT 21..27 = DG bits; wrong outputs) on
# the plain-epilogue shapes, one process per variant
set -o pipefail
for v in ${VARS:-10 21 22 23 24 25 26 27}; do
  timeout -k 10 200 env VTD_GEMM_VARIANT=$v python3 tools/gemm_bench.py --reps 10 --shapes ${SHAPES:-mlp2_noact,sq8192,mlp1_noact} >> gpurun_out/r2_diag.jsonl 2>/dev/null || exit 1
done
cat gpurun_out/r2_diag.jsonl
