#!/bin/bash
# Lockstep test (diagnostic library, VTD_PP2_SLEEP = s): first-round pp2 workgroups in odd XCD
# slots start s x 512 cycles late, so neighbouring CUs reach their epilogues (residual reads,
# output stores) out of step.  Per-shape gemm_bench times per s, interleaved, then the C2
# forward at s = 0 / best.
#   gpurun -- bash tools/experiments/r5_desync.sh <diag lib path> [shapes]
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$1
SH=${2:-attn_out_st,mlp3_st,qkv_ln,mlp1_ln,mlp2,attn_out_h,mlp3_h,head2}
O=$R/gpurun_out/desync; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for s in 0 4 8 16 32; do
    VTD_LIB_PATH=$D VTD_PP2_SLEEP=$s timeout -k 10 150 python tools/gemm_bench.py --shapes $SH > $O/g_s${s}_$r.log 2>&1 || { tail -5 $O/g_s${s}_$r.log; exit 1; }
    echo "r$r s=$s $(grep -o '"shape": "[a-z0-9_]*", "us": [0-9.]*' $O/g_s${s}_$r.log | sed 's/"shape": //; s/"us": //' | tr '\n' ' ')"
  done
done
for r in 1 2; do
  for s in 0 8 16; do
    VTD_LIB_PATH=$D VTD_PP2_SLEEP=$s timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 > $O/f_s${s}_$r.log 2>&1 || { tail -5 $O/f_s${s}_$r.log; exit 1; }
    echo "fwd r$r s=$s $(tail -1 $O/f_s${s}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
