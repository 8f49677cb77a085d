# quick A/B: GPU model tests subset + bench (default) + two-stream kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -k "two_stream or c2_b256 or graph" > gpurun_out/r2_quick_tests.log 2>&1 || { tail -30 gpurun_out/r2_quick_tests.log; exit 1; }
tail -2 gpurun_out/r2_quick_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_quick_bench.log 2>&1 || { tail -20 gpurun_out/r2_quick_bench.log; exit 1; }
tail -1 gpurun_out/r2_quick_bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r2_trace3 -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r2_trace3.log 2>&1 || exit 1
echo ok
