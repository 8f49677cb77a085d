set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 env VTD_GEMM_REF_LIB=1 python tools/gemm_bench.py > gpurun_out/r2_gemm_vendor.jsonl 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r2_trace1 -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --streams 1 > $R/gpurun_out/r2_trace1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r2_trace2 -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r2_trace2.log 2>&1 || exit 1
echo ok
