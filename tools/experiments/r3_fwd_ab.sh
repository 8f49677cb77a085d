#!/bin/bash
# round 3: forward A/B (C2 B=256 bf16): GEMM variant 10 (pp2) / 13 (w4 on residual-free layers, sched 1 / 2)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_fwd_ab2.log
for r in 1 2 3; do
  for v in "10 1" "13 1" "13 2"; do
    set -- $v
    VTD_GEMM_VARIANT=$1 VTD_W4_SCHED=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/b.json'));print('v$1 s$2', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'], d['roofline']['avg_launch_us'])" | tee -a $O
  done
done
