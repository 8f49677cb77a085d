#!/bin/bash
# Persistent attention at C2 (B=256), diag library VTD_ATTN_DMODE: 0 full, 8 multiply instead of
# exp2, 16 no V DMA, 24 both, 2 DMAs + stores only, 4 compute + stores only, 6 stores only;
# two passes over the modes.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/attn_dmode; mkdir -p $O
for pass in 1 2; do
for m in ${MODES:-0 8 16 24 2 4 6}; do
  VTD_LIB_PATH=$GRAFT_REPO_ROOT/vision_transformer_detector_amd/libvtd_diag.so VTD_ATTN_DMODE=$m \
    timeout -k 10 60 python tools/attn_bench.py --reps 50 --rounds 2 > $O/m${m}_$pass.log 2>&1 || exit 1
  echo "pass $pass mode $m: $(grep -o '"us": [0-9.]*' $O/m${m}_$pass.log | tr '\n' ' ')"
done
done
