#!/bin/bash
# round 3: streaming attention with the full chunks specialised at compile time (libvtd.so)
# vs before (libvtd_base.so): tests, then interleaved C3 / C5 forward A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py -m gpu -k "attention" > gpurun_out/r3_attn_last_tests.log 2>&1 || { tail -40 gpurun_out/r3_attn_last_tests.log; exit 1; }
tail -1 gpurun_out/r3_attn_last_tests.log
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_batch_parity.py -m gpu -k "c3 or c5" > gpurun_out/r3_attn_last_parity.log 2>&1 || { tail -30 gpurun_out/r3_attn_last_parity.log; exit 1; }
grep -i 'max-rel' gpurun_out/r3_attn_last_parity.log; tail -1 gpurun_out/r3_attn_last_parity.log
O=gpurun_out/r3_attn_last.log
run() {  # label, lib, bench args...
  local lab=$1; shift; local lib=$1; shift
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['mfma_util_attn_mlp'], d['kernels']['attention']['avg_us'], d['kernels']['attention']['tflops'])" | tee -a $O
}
for r in 1 2; do
  run c3_new libvtd --preset vit_b16_640 --batch 32 --steps 10 --warmup 3
  run c3_base libvtd_base --preset vit_b16_640 --batch 32 --steps 10 --warmup 3
done
run c5fp8_new libvtd --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3
run c5fp8_base libvtd_base --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3
run c5bf16_new libvtd --preset vit_l16_384 --batch 128 --steps 10 --warmup 3
run c5bf16_base libvtd_base --preset vit_l16_384 --batch 128 --steps 10 --warmup 3
