#!/bin/bash
# prev (libvtd_prev.so) vs new at C2 B = 256 and B = 64, 3 interleaved rounds; tests first
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab2}; K=$2; mkdir -p $O
P=$R/vision_transformer_detector_amd/libvtd_prev.so
export PYTHONUNBUFFERED=1
if [ -n "$K" ] && [ "$K" != "none" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for r in 1 2 3; do
  for b in 256 64; do
    VTD_LIB_PATH=$P timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 --batch $b > $O/p_b${b}_$r.log 2>&1 || { tail -5 $O/p_b${b}_$r.log; exit 1; }
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 --batch $b > $O/n_b${b}_$r.log 2>&1 || { tail -5 $O/n_b${b}_$r.log; exit 1; }
    echo "B=$b r$r prev $(tail -1 $O/p_b${b}_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/n_b${b}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
