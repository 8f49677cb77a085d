# Head join (VTD_HEAD_JOIN=1: the head's Dense chain once over the whole batch after the
# two-stream join): model / batch-parity tests with it, an interleaved forward A/B (default,
# join, join + split-K target 600), and the head section of a one-forward trace with the join.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c19
mkdir -p $O
VTD_HEAD_JOIN=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_batch_parity.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/def_$r.log 2>&1 || { tail -5 $O/def_$r.log; exit 1; }
  VTD_HEAD_JOIN=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/hj_$r.log 2>&1 || { tail -5 $O/hj_$r.log; exit 1; }
  VTD_HEAD_JOIN=1 VTD_SPLITK=600 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/hjs_$r.log 2>&1 || { tail -5 $O/hjs_$r.log; exit 1; }
  echo "r$r default $(tail -1 $O/def_$r.log | grep -o '"value": [0-9.]*') join $(tail -1 $O/hj_$r.log | grep -o '"value": [0-9.]*') join+splitk600 $(tail -1 $O/hjs_$r.log | grep -o '"value": [0-9.]*')"
done
cd /tmp && export TMPDIR=/tmp
export VTD_HEAD_JOIN=1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_hj -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/trace_hj.log 2>&1 || { tail -20 $O/trace_hj.log; exit 1; }
f=$(find $O/trace_hj -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_forward2.py $f 8 > $O/trace_summary_hj.txt 2>&1 || true
grep -A40 "head section" $O/trace_summary_hj.txt || true
