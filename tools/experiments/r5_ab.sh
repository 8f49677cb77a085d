#!/bin/bash
# round 5 A/B on one box: libvtd_prev.so (the previous commit's build) vs libvtd.so.
#   gpurun -- bash tools/experiments/r5_ab.sh <tag> "<pytest -k expr or empty>" "<gemm shapes>" <fwd rounds> [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r5ab}; K=$2; SH=${3:-attn_out_st,mlp3_st}; NR=${4:-2}; shift 4; BA="$@"
O=$R/gpurun_out/$T
mkdir -p $O
P=$R/vision_transformer_detector_amd/libvtd_prev.so
export PYTHONUNBUFFERED=1
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
if [ -n "$SH" ] && [ "$SH" != "none" ]; then
  for r in 1 2 3; do
    VTD_LIB_PATH=$P VTD_STAT_ROWMAJOR=1 timeout -k 10 120 python tools/gemm_bench.py --shapes $SH > $O/gemm_prev_$r.log 2>&1 || { tail -5 $O/gemm_prev_$r.log; exit 1; }
    timeout -k 10 120 python tools/gemm_bench.py --shapes $SH > $O/gemm_new_$r.log 2>&1 || { tail -5 $O/gemm_new_$r.log; exit 1; }
    echo "r$r prev: $(grep -o '"shape": "[a-z0-9_]*", "us": [0-9.]*' $O/gemm_prev_$r.log | tr '\n' ' ')"
    echo "r$r new : $(grep -o '"shape": "[a-z0-9_]*", "us": [0-9.]*' $O/gemm_new_$r.log | tr '\n' ' ')"
  done
fi
for r in $(seq 1 $NR); do
  VTD_LIB_PATH=$P timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 $BA > $O/fwd_prev_$r.log 2>&1 || { tail -5 $O/fwd_prev_$r.log; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 $BA > $O/fwd_new_$r.log 2>&1 || { tail -5 $O/fwd_new_$r.log; exit 1; }
  echo "fwd r$r prev $(tail -1 $O/fwd_prev_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/fwd_new_$r.log | grep -o '"value": [0-9.]*')"
done
echo done
