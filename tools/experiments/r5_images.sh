#!/bin/bash
# Same-box A/B of the headline's synthetic inputs: letterboxed U(-1, 1) images (the default,
# SURVEY 8(d) "COCO-shaped") against plain U(-1, 1) images, interleaved rounds.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/images; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for im in letterbox uniform; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 --images $im > $O/${im}_$r.log 2>&1 || { tail -5 $O/${im}_$r.log; exit 1; }
    echo "r$r $im $(tail -1 $O/${im}_$r.log | grep -o '"value": [0-9.]*\|"mfma_util_attn_mlp": [0-9.]*' | tr '\n' ' ')"
  done
done
