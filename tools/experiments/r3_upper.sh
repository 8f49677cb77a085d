#!/bin/bash
# round 3: split-K head (tests + forward A/B) and upper bounds in the C2 B=256 two-stream
# forward from the diag build (WRONG outputs, timing only): LayerNorm finalize launches
# skipped, attention skipped, head skipped.  Interleaved rounds on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_upper.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "splitk" > gpurun_out/r3_splitk_tests.log 2>&1 || { tail -30 gpurun_out/r3_splitk_tests.log; exit 1; }
tail -1 gpurun_out/r3_splitk_tests.log
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_batch_parity.py -m gpu -k "c2_b256 or c5" > gpurun_out/r3_splitk_parity.log 2>&1 || { tail -30 gpurun_out/r3_splitk_parity.log; exit 1; }
grep -i 'max-rel' gpurun_out/r3_splitk_parity.log; tail -1 gpurun_out/r3_splitk_parity.log
D=$R/vision_transformer_detector_amd/libvtd_diag.so
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['ms_per_step'], d['mfma_util_attn_mlp'])" | tee -a $O
}
for r in 1 2; do
  run splitk VTD_X=0
  run nosplitk VTD_SPLITK=0
  run nofin VTD_LIB_PATH=$D VTD_DIAG_NOFIN=1
  run noattn VTD_LIB_PATH=$D VTD_DIAG_NOATTN=1
  run nohead VTD_LIB_PATH=$D VTD_DIAG_NOHEAD=1
done
