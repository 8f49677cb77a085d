#!/bin/bash
# MX transposed kernel: default (activation layers without residual) vs knob GEMM_TR = 1 (also
# query/key/value, attention output is a residual layer: staged) vs 0 (none); C5 fp8 forward
# and gemm_bench_mx, interleaved; MX tests first.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/mxtr2; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "mx8 or mx" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for t in -1 1 0; do
    VTD_GEMM_TR=$t timeout -k 10 150 python tools/gemm_bench_mx.py --shapes qkv,mlp1,mlp2 > $O/g_t${t}_$r.log 2>&1 || { tail -5 $O/g_t${t}_$r.log; exit 1; }
    echo "r$r tr=$t $(grep -o '"us": [0-9.]*' $O/g_t${t}_$r.log | tr '\n' ' ')"
    VTD_GEMM_TR=$t timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --preset vit_l16_384 --batch 128 --dtype fp8 --steps 20 > $O/f_t${t}_$r.log 2>&1 || { tail -5 $O/f_t${t}_$r.log; exit 1; }
    echo "fwd r$r tr=$t $(tail -1 $O/f_t${t}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
