#!/bin/bash
# Persistent attention at C2 (B=256), diag library: full (0), loads + stores only (2),
# compute + stores only (4, no loads), head-major full (1); 3 rounds each, product first.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/attn_hm2; mkdir -p $O
timeout -k 10 60 python tools/attn_bench.py --reps 50 --rounds 3 > $O/prod.log 2>&1 || exit 1
echo "prod: $(grep -o '"us": [0-9.]*' $O/prod.log | tr '\n' ' ')"
for m in 0 2 4 1 0; do
  VTD_LIB_PATH=$GRAFT_REPO_ROOT/vision_transformer_detector_amd/libvtd_diag.so VTD_ATTN_DMODE=$m \
    timeout -k 10 60 python tools/attn_bench.py --reps 50 --rounds 3 > $O/m$m.log 2>&1 || exit 1
  echo "mode $m: $(grep -o '"us": [0-9.]*' $O/m$m.log | tr '\n' ' ')"
done
