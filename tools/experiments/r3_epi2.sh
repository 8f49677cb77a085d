#!/bin/bash
# round 3: rowadd / out2 epilogue bits (libvtd.so) vs HEAD (libvtd_base.so): C2 forward A/B,
# then the round-end evidence pass on libvtd.so (full GPU suite, bench, rocprof, PMC)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_epi2.log
run() {  # label, lib, bench args...
  local lab=$1; shift; local lib=$1; shift
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['mfma_util_attn_mlp'], d['roofline']['avg_launch_us'], d['kernels']['gemm']['tflops'])" | tee -a $O
}
for r in 1 2; do
  run c2_new libvtd --steps 20 --warmup 5
  run c2_base libvtd_base --steps 20 --warmup 5
done
bash tools/gpu_round_end.sh
