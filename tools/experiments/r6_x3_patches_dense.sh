# split-bf16 patch extraction on the dense (unpadded) kernel: tests, then bf16x3 one-stream kernel stats
set -o pipefail
O=gpurun_out/r6pd
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16x3.py tests/test_gpu_kernels.py tests/test_gpu_model.py -k "patches or bf16x3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 bench.py --dtype bf16x3 --streams 1 --steps 5 --warmup 2 --no-cpu-baseline --no-parity-mode > $O/prof.log 2>&1
grep -h "patches" $(find $O/raw -name '*kernel_stats.csv') | cut -c1-200
