# per-kernel time of the split-bf16 (bf16x3) forward, one stream, at the two-piece operand
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6x3prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6x3prof/raw -o run --output-format csv -- python3 bench.py --dtype bf16x3 --streams 1 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode > gpurun_out/r6x3prof/bench.log 2>&1
tail -1 gpurun_out/r6x3prof/bench.log
find gpurun_out/r6x3prof/raw -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r6x3prof/kernel_stats.csv
head -25 gpurun_out/r6x3prof/kernel_stats.csv | cut -c1-220
