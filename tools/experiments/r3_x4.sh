#!/bin/bash
# round 3: x4 MX-fp8 kernel: parity tests, then the C5 B=128 fp8 forward, MX variant 1 vs 2
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_x4.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mx8.py > gpurun_out/r3_x4_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3_x4_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 2; do
    VTD_MX_VARIANT=$v timeout -k 10 300 python -u bench.py --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/b.json'));k=d['kernels']['gemm'];print('c5 fp8 mx$v', d['value'], d['roofline']['frac'], k['avg_us'], k['tflops'])" | tee -a $O
  done
done
