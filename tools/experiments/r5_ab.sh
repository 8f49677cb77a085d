#!/bin/bash
# round 5 A/B on one box: libvtd_prev.so (the previous commit's build) vs libvtd.so.
#   gpurun -- bash tools/experiments/r5_ab.sh <tag> "<pytest -k expr | none>" "<micro command | none>" <fwd rounds> [bench args]
# micro command: run 3 times per library, interleaved (e.g. "python tools/attn_bench.py")
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r5ab}; K=$2; MC=$3; NR=${4:-2}; shift 4; BA="$@"
O=$R/gpurun_out/$T
mkdir -p $O
P=$R/vision_transformer_detector_amd/libvtd_prev.so
export PYTHONUNBUFFERED=1
if [ -n "$K" ] && [ "$K" != "none" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
if [ -n "$MC" ] && [ "$MC" != "none" ]; then
  for r in 1 2 3; do
    VTD_LIB_PATH=$P timeout -k 10 120 $MC > $O/micro_prev_$r.log 2>&1 || { tail -5 $O/micro_prev_$r.log; exit 1; }
    timeout -k 10 120 $MC > $O/micro_new_$r.log 2>&1 || { tail -5 $O/micro_new_$r.log; exit 1; }
    echo "r$r prev: $(grep -o '"[a-z_]*": "[a-z0-9_]*", "us": [0-9.]*\|"us": [0-9.]*' $O/micro_prev_$r.log | tr '\n' ' ')"
    echo "r$r new : $(grep -o '"[a-z_]*": "[a-z0-9_]*", "us": [0-9.]*\|"us": [0-9.]*' $O/micro_new_$r.log | tr '\n' ' ')"
  done
fi
for r in $(seq 1 $NR); do
  VTD_LIB_PATH=$P timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 $BA > $O/fwd_prev_$r.log 2>&1 || { tail -5 $O/fwd_prev_$r.log; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 $BA > $O/fwd_new_$r.log 2>&1 || { tail -5 $O/fwd_new_$r.log; exit 1; }
  echo "fwd r$r prev $(tail -1 $O/fwd_prev_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/fwd_new_$r.log | grep -o '"value": [0-9.]*')"
done
echo done
