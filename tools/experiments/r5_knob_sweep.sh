#!/bin/bash
# Knob sweep on the non-headline configs (C5 fp8 B=128, C3 B=32): the defaults were tuned on
# C2.  Interleaved, 2 rounds; env knobs only (no rebuild).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/knobs; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for cfg in "c5fp8:--preset vit_l16_384 --batch 128 --dtype fp8" "c3:--preset vit_b16_640 --batch 32"; do
    lab=${cfg%%:*}; args=${cfg#*:}
    for kn in "base:" "ngw2:VTD_GEMM_NGW=2" "ngw8:VTD_GEMM_NGW=8" "stag1:VTD_STAGGER=1" "nopad:VTD_SPLIT_PAD=0"; do
      kl=${kn%%:*}; ke=${kn#*:}
      env $ke timeout -k 10 150 python bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3 $args > $O/${lab}_${kl}_$r.log 2>&1 || { tail -5 $O/${lab}_${kl}_$r.log; exit 1; }
      echo "r$r $lab $kl $(tail -1 $O/${lab}_${kl}_$r.log | grep -o '"value": [0-9.]*')"
    done
  done
done
