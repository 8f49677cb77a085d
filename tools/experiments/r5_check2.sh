#!/bin/bash
# round 5: attention (trimmed last block, long-sequence LDS-DMA kernel) + residual LDS prefetch
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5c2; mkdir -p $O
P=$R/vision_transformer_detector_amd/libvtd_prev.so
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or statout or batched_forward_matches_golden and (c2_b256 or c3_b32 or c5_b128) and bfloat16" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for lib in prev new; do
    if [ $lib = prev ]; then export VTD_LIB_PATH=$P; else unset VTD_LIB_PATH; fi
    timeout -k 10 100 python tools/attn_bench.py --rounds 1 > $O/attn_c2_${lib}_$r.log 2>&1 || exit 1
    timeout -k 10 100 python tools/attn_bench.py --rounds 1 --B 32 --N 1600 > $O/attn_c3_${lib}_$r.log 2>&1 || exit 1
    timeout -k 10 100 python tools/attn_bench.py --rounds 1 --B 128 --N 576 --H 16 > $O/attn_c5_${lib}_$r.log 2>&1 || exit 1
    timeout -k 10 100 python tools/gemm_bench.py --shapes attn_out_st,mlp3_st > $O/gemm_${lib}_$r.log 2>&1 || exit 1
    echo "r$r $lib c2 $(grep -o '"us": [0-9.]*' $O/attn_c2_${lib}_$r.log | tr '\n' ' ') c3 $(grep -o '"us": [0-9.]*' $O/attn_c3_${lib}_$r.log | tr '\n' ' ') c5 $(grep -o '"us": [0-9.]*' $O/attn_c5_${lib}_$r.log | tr '\n' ' ') gemm $(grep -o '"us": [0-9.]*' $O/gemm_${lib}_$r.log | tr '\n' ' ')"
  done
done
unset VTD_LIB_PATH
for r in 1 2; do
  VTD_LIB_PATH=$P timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 > $O/fwd_prev_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 > $O/fwd_new_$r.log 2>&1 || exit 1
  VTD_LIB_PATH=$P timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --preset vit_b16_640 --batch 32 --steps 10 > $O/c3_prev_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --preset vit_b16_640 --batch 32 --steps 10 > $O/c3_new_$r.log 2>&1 || exit 1
  echo "fwd r$r prev $(tail -1 $O/fwd_prev_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/fwd_new_$r.log | grep -o '"value": [0-9.]*')  C3 prev $(tail -1 $O/c3_prev_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/c3_new_$r.log | grep -o '"value": [0-9.]*')"
done
echo done
