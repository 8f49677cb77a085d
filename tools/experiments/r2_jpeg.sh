set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/jpeg_bench.py > gpurun_out/r2_jpeg_bench.json 2>/dev/null || exit 1
cat gpurun_out/r2_jpeg_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/jpeg_prof -o p --output-format csv -- python3 $R/tools/jpeg_bench.py --reps 3 > /dev/null 2>&1 || exit 1
echo ok
