#!/bin/bash
# round 5: long-sequence attention kernel configurations vs the streaming kernel (knob 2/4 default)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fl; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "long_sequence" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in "-1 0" "6 0" "6 1" "6 2"; do
    set -- $v
    VTD_ATTN_VARIANT=$1 VTD_FL_CFG=$2 timeout -k 10 100 python tools/attn_bench.py --rounds 1 --B 32 --N 1600 > $O/c3_$1_$2_$r.log 2>&1 || exit 1
    VTD_ATTN_VARIANT=$1 VTD_FL_CFG=$2 timeout -k 10 100 python tools/attn_bench.py --rounds 1 --B 128 --N 576 --H 16 > $O/c5_$1_$2_$r.log 2>&1 || exit 1
    echo "r$r variant $1 cfg $2: c3 $(grep -o '"us": [0-9.]*' $O/c3_$1_$2_$r.log) c5 $(grep -o '"us": [0-9.]*' $O/c5_$1_$2_$r.log)"
  done
done
