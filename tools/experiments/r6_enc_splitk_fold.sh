# bf16 small batches: the LayerNorm-fold layers (query/key/value, first MLP) split K too
set -o pipefail
O=gpurun_out/r6ef
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "splitk or fold" tests/test_gpu_model.py tests/test_gpu_batch_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for b in 1 8 16 32 64; do
  for es in 0 1; do
    VTD_ENC_SPLITK=$es timeout -k 10 300 python bench.py --dtype bf16 --batch $b --steps 20 --warmup 5 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16 b=$b enc_splitk=$es', d['value'], 'img/s', d['ms_per_step'], 'ms')" || exit 1
  done
done
