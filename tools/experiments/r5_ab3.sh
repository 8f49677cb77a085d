#!/bin/bash
# three-way A/B on one box: libvtd_prev.so, libvtd_mid.so, libvtd.so (interleaved).
#   gpurun -- bash tools/experiments/r5_ab3.sh <tag> "<pytest -k expr | none>" "<micro command | none>" <fwd rounds> [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r5ab3}; K=$2; MC=$3; NR=${4:-2}; shift 4; BA="$@"
O=$R/gpurun_out/$T
mkdir -p $O
D=$R/vision_transformer_detector_amd
export PYTHONUNBUFFERED=1
if [ -n "$K" ] && [ "$K" != "none" ]; then
  for L in mid new; do
    LP=$D/libvtd.so; [ $L = mid ] && LP=$D/libvtd_mid.so
    VTD_LIB_PATH=$LP timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $O/tests_$L.log 2>&1 || { tail -30 $O/tests_$L.log; exit 1; }
    echo "tests $L: $(tail -1 $O/tests_$L.log)"
  done
fi
for r in $(seq 1 $NR); do
  for L in prev mid new; do
    LP=$D/libvtd.so; [ $L != new ] && LP=$D/libvtd_$L.so
    if [ -n "$MC" ] && [ "$MC" != "none" ]; then
      VTD_LIB_PATH=$LP timeout -k 10 120 $MC > $O/micro_${L}_$r.log 2>&1 || { tail -5 $O/micro_${L}_$r.log; exit 1; }
      echo "r$r $L micro: $(grep -o '"shape": "[a-z0-9_]*", "us": [0-9.]*' $O/micro_${L}_$r.log | sed 's/"shape": //;s/"us": //' | tr '\n' ' ')"
    fi
    VTD_LIB_PATH=$LP timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 $BA > $O/fwd_${L}_$r.log 2>&1 || { tail -5 $O/fwd_${L}_$r.log; exit 1; }
    echo "fwd r$r $L $(tail -1 $O/fwd_${L}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
