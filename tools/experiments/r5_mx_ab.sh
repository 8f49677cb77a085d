#!/bin/bash
# prev (libvtd_prev.so) vs new MX-fp8 GEMM: MX tests + the C5 fp8 golden, gemm_bench_mx per C5
# shape interleaved, then the C5 fp8 forward interleaved (3 rounds each).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-mx_ab}; mkdir -p $O
P=$R/vision_transformer_detector_amd/libvtd_prev.so
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "mx8 or fp8 or float8" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  VTD_LIB_PATH=$P timeout -k 10 120 python tools/gemm_bench_mx.py --variants 1 --reps 10 --shapes qkv,attn_out,mlp1,mlp2,mlp3,sq8192 > $O/g_p$r.log 2>&1 || exit 1
  timeout -k 10 120 python tools/gemm_bench_mx.py --variants 1 --reps 10 --shapes qkv,attn_out,mlp1,mlp2,mlp3,sq8192 > $O/g_n$r.log 2>&1 || exit 1
  echo "r$r prev: $(grep -o '"us": [0-9.]*' $O/g_p$r.log | tr '\n' ' ')"
  echo "r$r new : $(grep -o '"us": [0-9.]*' $O/g_n$r.log | tr '\n' ' ')"
done
for r in 1 2 3; do
  VTD_LIB_PATH=$P timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 > $O/p_$r.log 2>&1 || { tail -5 $O/p_$r.log; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 > $O/n_$r.log 2>&1 || { tail -5 $O/n_$r.log; exit 1; }
  echo "fwd r$r prev $(tail -1 $O/p_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/n_$r.log | grep -o '"value": [0-9.]*')"
done
