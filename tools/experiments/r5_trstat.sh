#!/bin/bash
# Residual-layer GEMMs with / without the LayerNorm partial statistics, transposed (TR = 1) or
# staged (TR = 0) accumulator epilogue (knob VTD_GEMM_TR), gemm_bench per launch, interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/trstat; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for t in -1 0 1; do
    VTD_GEMM_TR=$t timeout -k 10 150 python tools/gemm_bench.py --shapes attn_out_st,attn_out,mlp3_st,mlp3,attn_out_h,mlp3_h --reps 30 > $O/t${t}_$r.log 2>&1 || { tail -5 $O/t${t}_$r.log; exit 1; }
    echo "r$r tr=$t $(grep -o '"shape": "[a-z0-9_]*", "us": [0-9.]*' $O/t${t}_$r.log | sed 's/"shape": //; s/"us": //' | tr '\n' ' ')"
  done
done
