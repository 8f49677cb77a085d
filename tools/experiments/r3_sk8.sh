#!/bin/bash
# round 3: vectorised split-K reduce/epilogue for the head (libvtd.so) vs HEAD (libvtd_base.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "splitk" > gpurun_out/r3_sk8_tests.log 2>&1 || { tail -30 gpurun_out/r3_sk8_tests.log; exit 1; }
tail -1 gpurun_out/r3_sk8_tests.log
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_batch_parity.py -m gpu -k "bfloat16" > gpurun_out/r3_sk8_parity.log 2>&1 || { tail -30 gpurun_out/r3_sk8_parity.log; exit 1; }
grep -i 'max-rel' gpurun_out/r3_sk8_parity.log; tail -1 gpurun_out/r3_sk8_parity.log
O=gpurun_out/r3_sk8.log
run() {  # label, lib
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/$2.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$1', d['value'], d['mfma_util_attn_mlp'], d['roofline']['avg_launch_us'])" | tee -a $O
}
for r in 1 2 3; do
  run c2_new libvtd
  run c2_base libvtd_base
done
