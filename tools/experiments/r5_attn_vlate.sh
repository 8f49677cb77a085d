#!/bin/bash
# Persistent attention with V waited for after the scores (prev = libvtd_prev.so): attention
# tests, attn_bench prev / new interleaved, then the C2 forward A/B (r5_ab2.sh without tests).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-vlate}; mkdir -p $O
P=$R/vision_transformer_detector_amd/libvtd_prev.so
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or batch_parity or two_stream" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  VTD_LIB_PATH=$P timeout -k 10 60 python tools/attn_bench.py --reps 50 > $O/attn_p$r.log 2>&1 || exit 1
  timeout -k 10 60 python tools/attn_bench.py --reps 50 > $O/attn_n$r.log 2>&1 || exit 1
  echo "attn r$r prev $(grep -o '"us": [0-9.]*' $O/attn_p$r.log) new $(grep -o '"us": [0-9.]*' $O/attn_n$r.log)"
done
bash $R/tools/experiments/r5_ab2.sh ${1:-vlate}_ab none
