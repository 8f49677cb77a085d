#!/bin/bash
# round 3: wide LayerNorm (parity tests), C5 fp8 forward, C2 forward
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mx8.py tests/test_gpu_kernels.py -k "layernorm or ln_ or mx8 or stats" 2>&1 | tail -2 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_batch_parity.py 2>&1 | tail -2 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));k=d['kernels'];print('c5 fp8', d['value'], d['roofline']['frac'], k['gemm']['avg_us'], k['layernorm']['avg_us'])" | tee -a gpurun_out/r3_ln.log
done
timeout -k 10 300 python -u bench.py --dtype f32 --batch 256 --steps 5 --warmup 2 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('/tmp/b.json'));k=d['kernels'];print('c2 f32', d['value'], d['mfma_util_attn_mlp'], k['layernorm']['avg_us'])" | tee -a gpurun_out/r3_ln.log
