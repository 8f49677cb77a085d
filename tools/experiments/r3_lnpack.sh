#!/bin/bash
# round 3: MX-fp8 LayerNorm with dword scale stores (parity tests), C5 fp8 forward A/B vs the
# previous library (libvtd_base.so, byte scale stores), interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_lnpack.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mx8.py tests/test_gpu_kernels.py -k "layernorm or ln_ or mx8" > gpurun_out/r3_lnpack_tests.log 2>&1 || { tail -30 gpurun_out/r3_lnpack_tests.log; exit 1; }
tail -2 gpurun_out/r3_lnpack_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch_parity.py -k "c5_b128" > gpurun_out/r3_lnpack_parity.log 2>&1 || { tail -30 gpurun_out/r3_lnpack_parity.log; exit 1; }
tail -2 gpurun_out/r3_lnpack_parity.log
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_base.so; else unset VTD_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/b.json'));k=d['kernels'];print('c5 fp8 $v', d['value'], d['roofline']['frac'], k['gemm']['avg_us'], k['layernorm']['avg_us'])" | tee -a $O
  done
done
