#!/bin/bash
# round 3: compile-time LayerNorm-fold / statistics / fp8-out epilogue bits (libvtd.so) vs
# runtime checks (libvtd_base.so): GEMM / model tests + goldens, then interleaved forward A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py -m gpu -k "gemm or statout or layernorm or fold or mx8" > gpurun_out/r3_epi_tests.log 2>&1 || { tail -40 gpurun_out/r3_epi_tests.log; exit 1; }
tail -1 gpurun_out/r3_epi_tests.log
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_batch_parity.py tests/test_gpu_model.py -m gpu > gpurun_out/r3_epi_parity.log 2>&1 || { tail -30 gpurun_out/r3_epi_parity.log; exit 1; }
grep -i 'max-rel' gpurun_out/r3_epi_parity.log; tail -1 gpurun_out/r3_epi_parity.log
O=gpurun_out/r3_epi.log
run() {  # label, lib, bench args...
  local lab=$1; shift; local lib=$1; shift
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['mfma_util_attn_mlp'], d['roofline']['avg_launch_us'], d['kernels']['gemm']['tflops'])" | tee -a $O
}
for r in 1 2 3; do
  run c2_new libvtd --steps 20 --warmup 5
  run c2_base libvtd_base --steps 20 --warmup 5
done
run c5fp8_new libvtd --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3
run c5fp8_base libvtd_base --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3
