#!/bin/bash
# round 3 (final kernels): GEMM tile-order group width override (VTD_GEMM_NGW, all GEMMs) vs
# the default per-shape choice, C2 B=256 forward, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_ngw.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['mfma_util_attn_mlp'], d['roofline']['avg_launch_us'])" | tee -a $O
}
for r in 1 2; do
  run default VTD_X=0
  run ngw2 VTD_GEMM_NGW=2
  run ngw3 VTD_GEMM_NGW=3
  run ngw6 VTD_GEMM_NGW=6
  run ngw0 VTD_GEMM_NGW=0
done
