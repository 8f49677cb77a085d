#!/bin/bash
# round 3: fused LayerNorm finalize kernel test + determinism, then the forward A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "gemm_ln or splitk or statout or layernorm_fold" > gpurun_out/r3_fin_tests.log 2>&1 || { tail -40 gpurun_out/r3_fin_tests.log; exit 1; }
tail -1 gpurun_out/r3_fin_tests.log
timeout -k 10 200 python -u tools/r3_determinism.py 128 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_det.log
O=gpurun_out/r3_fin.log
D=$R/vision_transformer_detector_amd/libvtd_diag.so
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['ms_per_step'], d['mfma_util_attn_mlp'])" | tee -a $O
}
for r in 1 2; do
  run fused VTD_X=0
  run finlaunch VTD_LN_FINALIZE=1
  run nofin240 VTD_LIB_PATH=$D VTD_DIAG_NOFIN=240 VTD_LN_FINALIZE=1
  run attngrid512 VTD_ATTN_GRID=512
  run attngrid768 VTD_ATTN_GRID=768
  run attngrid1536 VTD_ATTN_GRID=1536
done
