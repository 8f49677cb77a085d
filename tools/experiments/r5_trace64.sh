#!/bin/bash
# Kernel traces of C2 at B = 64: two padded parts (VTD_SPLIT_MIN_TILES=24) and one stream
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace64; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
VTD_SPLIT_MIN_TILES=24 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/split -o p --output-format csv -- python3 $R/bench.py --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode > $O/split.log 2>&1 || { tail -20 $O/split.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/one -o p --output-format csv -- python3 $R/bench.py --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode > $O/one.log 2>&1 || { tail -20 $O/one.log; exit 1; }
cd $R
for t in split one; do
  f=$(find $O/$t -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_forward2.py $f 8 $([ $t = split ] && echo 2 || echo 1) > $O/$t.summary.txt 2>&1 || true
  head -30 $O/$t.summary.txt
done
