#!/bin/bash
# round 3: C2 B=64 with the batch split over 1-4 streams (VTD_STREAMS, VTD_SPLIT_MIN_TILES)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_split.log
for r in 1 2; do
  for s in 1 2 3 4; do
    VTD_STREAMS=$s VTD_SPLIT_MIN_TILES=8 timeout -k 10 200 python -u bench.py --batch 64 --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/b.json'));print('b64 streams $s', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'])" | tee -a $O
  done
done
for s in 2 3 4; do
  VTD_STREAMS=$s timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('b256 streams $s', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'])" | tee -a $O
done
