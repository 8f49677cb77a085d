#!/bin/bash
# uneven two-stream split (VTD_SPLIT_P0 = part 0's share in per mille), interleaved rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/skew; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for p in 0 480 460 440 420; do
    VTD_SPLIT_P0=$p timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 "$@" > $O/p${p}_$r.log 2>&1 || { tail -5 $O/p${p}_$r.log; exit 1; }
    echo "r$r p0=$p $(tail -1 $O/p${p}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
