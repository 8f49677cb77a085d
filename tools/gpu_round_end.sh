# Round-end evidence on the GPU box: full -m gpu suite (batched parity errors printed),
# headline bench line, rocprofv3 kernel-trace stats of the same bench command (one stream
# and default), PMC FETCH/WRITE passes for `traffic`, per-mode accuracy of the goldens.
#   gpurun --timeout 1200 -- bash tools/gpu_round_end.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 200 python tools/accuracy_report.py --out gpurun_out/accuracy.json > gpurun_out/accuracy.log 2>&1 || { tail -20 gpurun_out/accuracy.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
# kernel evidence on one stream (--streams 1: every launch alone, as in bench.py's profiled
# pass that the roofline object comes from); then the default two-stream command
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 1 > $R/gpurun_out/prof.log 2>&1 || { tail -20 $R/gpurun_out/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2 -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof2.log 2>&1 || { tail -20 $R/gpurun_out/prof2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --streams 1 > $R/gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --streams 1 > $R/gpurun_out/pmc_write.log 2>&1 || exit 1
echo done
