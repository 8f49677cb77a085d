# kernel traces (one stream) with the small-GEMM kernel off / on: the head's dispatches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for g in 0 1; do
  VTD_GEMM_SMALL=$g timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/strace_$g -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams 1 > $R/gpurun_out/strace_$g.log 2>&1 || { tail -5 $R/gpurun_out/strace_$g.log; exit 1; }
done
echo ok
