# rocprofv3 kernel-trace stats of a short bench run (gpurun -- bash tools/prof_stats.sh [bench args])
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $R/gpurun_out/prof.log 2>&1 || { tail -20 $R/gpurun_out/prof.log; exit 1; }
tail -1 $R/gpurun_out/prof.log
f=$(find $R/gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -14
