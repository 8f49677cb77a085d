#!/bin/bash
# round 3: persistent-attention grid A/B in the C2 B=256 two-stream forward (more workgroups
# than CUs: a workgroup that starts late, on a CU the other stream's GEMM just freed, holds
# fewer pairs) + split-K off; then one default kernel trace for the head / overlap analysis
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -k "splitk or statout or layernorm or attention or two_stream or removed" > gpurun_out/r3_grid_tests.log 2>&1 || { tail -40 gpurun_out/r3_grid_tests.log; exit 1; }
tail -1 gpurun_out/r3_grid_tests.log
O=gpurun_out/r3_grid.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['ms_per_step'], d['mfma_util_attn_mlp'])" | tee -a $O
}
for r in 1 2; do
  run base VTD_X=0
  run grid384 VTD_ATTN_GRID=384
  run grid512 VTD_ATTN_GRID=512
  run splitk0 VTD_SPLITK=0
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof3 -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof3.log 2>&1 || { tail -20 $R/gpurun_out/prof3.log; exit 1; }
echo done
