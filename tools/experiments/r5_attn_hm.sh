#!/bin/bash
# Persistent attention at C2 (B=256): diagnostic modes of the diag library (VTD_ATTN_DMODE
# bit 0 head-major Q/K/V reads, bit 1 loads + stores only), with and without MALL eviction.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/attn_hm; mkdir -p $O
timeout -k 10 60 python tools/attn_bench.py --reps 20 --rounds 2 > $O/prod.log 2>&1 || exit 1
cat $O/prod.log
for m in 0 1 2 3; do
  for f in "" "--flush"; do
    VTD_LIB_PATH=$GRAFT_REPO_ROOT/vision_transformer_detector_amd/libvtd_diag.so VTD_ATTN_DMODE=$m \
      timeout -k 10 60 python tools/attn_bench.py --reps 20 --rounds 2 $f > $O/m$m$f.log 2>&1 || exit 1
    echo "mode $m $f: $(tail -1 $O/m$m$f.log)"
  done
done
