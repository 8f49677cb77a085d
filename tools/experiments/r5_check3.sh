#!/bin/bash
# full -m gpu suite, the headline bench line, one default (two-stream) kernel trace + its
# one-forward summary (head section)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof2 -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
cd $R
f=$(find $O/prof2 -name '*kernel_trace.csv' | head -1)
python3 tools/trace_forward2.py $f 8 2 > $O/trace_summary.txt 2>&1 || true
cat $O/trace_summary.txt
rm -f $f
