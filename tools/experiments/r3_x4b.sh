#!/bin/bash
# round 3: x4 (sched 1 / 2) vs ping-pong MX GEMM per C5 shape, x4 diagnostics (diag lib:
# no DMA / no epilogue), C5 fp8 forward per variant, the MX tests
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_x4b.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mx8.py 2>&1 | tail -2 || exit 1
timeout -k 10 300 python -u tools/gemm_bench_mx.py --variants 1,2 | tee $O || exit 1
VTD_X4_SCHED=1 timeout -k 10 300 python -u tools/gemm_bench_mx.py --variants 2 | sed 's/"variant": "2"/"variant": "2s1"/' | tee -a $O || exit 1
for dg in 1 2 3; do
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_diag.so VTD_X4_DG=$dg timeout -k 10 300 python -u tools/gemm_bench_mx.py --variants 2 --shapes qkv,mlp2,sq8192 | tee -a $O || exit 1
done
for v in 1 2; do
  VTD_MX_VARIANT=$v timeout -k 10 300 python -u bench.py --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));k=d['kernels'];print('c5 fp8 mx$v', d['value'], d['roofline']['frac'], k['gemm']['avg_us'], k['layernorm']['avg_us'])" | tee -a gpurun_out/r3_x4b.log
done
