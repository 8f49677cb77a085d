# pp3 persistent (variant 11) vs pp2 (10) with the problem split in two concurrent M-halves;
# pp3 grid 256 and 128 (VTD_PP3_GRID) -- shapes without a bf16 residual
set -o pipefail
for cfg in "10 0" "11 0" "11 128" "10 0" "11 128"; do
  set -- $cfg
  if [ "$2" = "0" ]; then unset VTD_PP3_GRID; else export VTD_PP3_GRID=$2; fi
  VTD_GEMM_SPLIT2=1 VTD_GEMM_VARIANT=$1 timeout -k 10 200 python3 tools/gemm_bench.py --reps 10 --shapes qkv,mlp1,mlp2 2>/dev/null | sed "s/^/v$1 grid$2 /" || exit 1
done
