#!/bin/bash
# Head split-K target per launch beyond 256 (VTD_SPLITK >= 64 = the target): more splits for
# head2 (153 tiles per part, 136 K-steps); C2 B = 256, interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/splitk2; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for k in -1 256 384 512 768; do
    VTD_SPLITK=$k timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 > $O/b256_sk${k}_$r.log 2>&1 || { tail -5 $O/b256_sk${k}_$r.log; exit 1; }
    echo "b256 r$r sk=$k $(tail -1 $O/b256_sk${k}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
