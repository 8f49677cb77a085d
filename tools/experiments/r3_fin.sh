#!/bin/bash
# round 3: LayerNorm finalize fused into the consumer pp2 GEMM vs the separate finalize
# launch (VTD_LN_FINALIZE=1) vs no finalize at all (diag build, every finalize after the
# first 240 skipped: the consumers keep the last real statistics, activations stay
# realistic).  C2 B=256 two-stream forward, interleaved rounds on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_fin.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "statout or finalize or layernorm or splitk" > gpurun_out/r3_fin_tests.log 2>&1 || { tail -30 gpurun_out/r3_fin_tests.log; exit 1; }
tail -1 gpurun_out/r3_fin_tests.log
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_batch_parity.py -m gpu -k "fused_layernorm or c2_b256 or c5_b128 or two_stream" > gpurun_out/r3_fin_parity.log 2>&1 || { tail -30 gpurun_out/r3_fin_parity.log; exit 1; }
grep -i 'max-rel' gpurun_out/r3_fin_parity.log; tail -1 gpurun_out/r3_fin_parity.log
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
done
