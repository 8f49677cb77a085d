# Skinny kernel for the head's Dense(544) too (knob VTD_SKINNY=640: N threshold 640, that layer
# no longer split-K): model tests with it, an interleaved forward A/B, and the head section of a
# one-forward kernel trace each way.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c18
mkdir -p $O
VTD_SKINNY=640 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_batch_parity.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/def_$r.log 2>&1 || { tail -5 $O/def_$r.log; exit 1; }
  VTD_SKINNY=640 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/sk_$r.log 2>&1 || { tail -5 $O/sk_$r.log; exit 1; }
  echo "r$r default $(tail -1 $O/def_$r.log | grep -o '"value": [0-9.]*') skinny640 $(tail -1 $O/sk_$r.log | grep -o '"value": [0-9.]*')"
done
cd /tmp && export TMPDIR=/tmp
for v in def sk; do
  if [ $v = sk ]; then export VTD_SKINNY=640; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$v -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/trace_$v.log 2>&1 || { tail -20 $O/trace_$v.log; exit 1; }
  f=$(find $O/trace_$v -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_forward2.py $f 8 > $O/trace_summary_$v.txt 2>&1 || true
  grep -A3 "head section" $O/trace_summary_$v.txt || true
done
