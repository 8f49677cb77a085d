#!/bin/bash
# Persistent attention grid per launch (VTD_ATTN_GRID; default one workgroup per CU) with the
# two micro-batch parts' attention launches co-running; C2 B = 256 and 64, interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/attngrid; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for gsz in -1 128 192; do
    for b in 256 64; do
      VTD_ATTN_GRID=$gsz timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 --batch $b > $O/b${b}_g${gsz}_$r.log 2>&1 || { tail -5 $O/b${b}_g${gsz}_$r.log; exit 1; }
      echo "b$b r$r grid=$gsz $(tail -1 $O/b${b}_g${gsz}_$r.log | grep -o '"value": [0-9.]*')"
    done
  done
done
