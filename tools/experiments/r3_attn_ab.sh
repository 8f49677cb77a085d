#!/bin/bash
# round 3: attention A/B (libvtd_base.so = before, libvtd.so = after), interleaved rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_attn_ab.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "attention" > gpurun_out/r3_attn_tests.log 2>&1 || { tail -20 gpurun_out/r3_attn_tests.log; exit 1; }
tail -1 gpurun_out/r3_attn_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch_parity.py -m gpu -k "c2_b256" > gpurun_out/r3_attn_parity.log 2>&1 || { tail -20 gpurun_out/r3_attn_parity.log; exit 1; }
tail -1 gpurun_out/r3_attn_parity.log
for r in 1 2 3; do
  for lib in libvtd_base libvtd; do
    VTD_LIB_PATH=$R/vision_transformer_detector_amd/$lib.so timeout -k 10 100 python -u tools/attn_bench.py --reps 30 | sed "s/^/$lib /" | tee -a $O || exit 1
  done
done
for r in 1 2; do
  for lib in libvtd_base libvtd; do
    VTD_LIB_PATH=$R/vision_transformer_detector_amd/$lib.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lib fwd', d['value'], d['mfma_util_attn_mlp'], d['kernels']['attention']['avg_us'])" | tee -a $O
  done
done
