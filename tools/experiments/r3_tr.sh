#!/bin/bash
# round 3: transposed-accumulator (register-direct) epilogue for every GEMM vs for the
# activation layers only, with the specialised epilogues (C2 B=256 forward, interleaved)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "gemm or statout or fold" > gpurun_out/r3_tr_tests.log 2>&1 || { tail -30 gpurun_out/r3_tr_tests.log; exit 1; }
VTD_GEMM_TR=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "gemm or statout or fold" > gpurun_out/r3_tr_tests1.log 2>&1 || { tail -30 gpurun_out/r3_tr_tests1.log; exit 1; }
tail -1 gpurun_out/r3_tr_tests.log; tail -1 gpurun_out/r3_tr_tests1.log
O=gpurun_out/r3_tr.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['mfma_util_attn_mlp'], d['roofline']['avg_launch_us'])" | tee -a $O
}
for r in 1 2 3; do
  run tr_act VTD_X=0
  run tr_all VTD_GEMM_TR=1
done
