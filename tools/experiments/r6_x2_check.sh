# two-piece split-bf16 A operand ([hi | lo], the GEMM K loop wraps A): the split-bf16 kernel
# tests, the bf16x3 model / batch goldens, then bf16x3 and bf16 bench lines, twice each
set -o pipefail
O=gpurun_out/r6x2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bf16x3.py tests/test_gpu_model.py tests/test_gpu_batch_parity.py tests/test_gpu_kernels.py \
  -k "split or bf16x3 or splitk" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype bf16x3 --no-cpu-baseline --no-parity-mode > $O/b3_$i.log 2>&1 || exit 1
  tail -1 $O/b3_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16x3', d['value'], d['ms_per_step'])"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-mode > $O/b16_$i.log 2>&1 || exit 1
  tail -1 $O/b16_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16', d['value'], d['ms_per_step'])"
done
