# split-bf16 skinny GEMM (Bt staged as [hi | lo]): split tests, then bf16x3 and bf16 lines
set -o pipefail
O=gpurun_out/r6sk
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bf16x3.py tests/test_gpu_model.py tests/test_gpu_kernels.py tests/test_gpu_batch_parity.py \
  -k "split or bf16x3 or splitk or skinny or gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype bf16x3 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16x3', d['value'], d['ms_per_step'])" || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16', d['value'], d['ms_per_step'])" || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/raw -o run --output-format csv -- python3 bench.py --dtype bf16x3 --streams 1 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode > $O/prof.log 2>&1
cp $O/raw/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || find $O/raw -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
