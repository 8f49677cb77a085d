#!/bin/bash
# round 3: forward A/B (C2 B=256 bf16): GEMM variant 12 (w4, sched 1 / 2) vs 10 (pp2), interleaved rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_fwd_ab.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch_parity.py -m gpu -k "c2_b256" > gpurun_out/r3_fwd_parity.log 2>&1 || { tail -20 gpurun_out/r3_fwd_parity.log; exit 1; }
tail -1 gpurun_out/r3_fwd_parity.log
for r in 1 2; do
  for v in "12 1" "12 2" "10 1"; do
    set -- $v
    VTD_GEMM_VARIANT=$1 VTD_W4_SCHED=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/b.json'));print('v$1 s$2', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'], d['roofline']['avg_launch_us'])" | tee -a $O
  done
done
