#!/bin/bash
# round 3: micro-batch side-stream priority A/B (C2 B=256 two-stream forward)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_prio.log
python3 -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');lo=ctypes.c_int();hi=ctypes.c_int();print('priority range', h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo),ctypes.byref(hi)), lo.value, hi.value)" | tee -a $O
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('$lab', d['value'], d['ms_per_step'], d['mfma_util_attn_mlp'])" | tee -a $O
}
for r in 1 2; do
  run base VTD_X=0
  run side_high VTD_SIDE_PRIORITY=high
  run side_low VTD_SIDE_PRIORITY=low
done
