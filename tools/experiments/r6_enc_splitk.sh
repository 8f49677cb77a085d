# split-K for the encoder's few-tile long-K Dense layers (small batches; default now) vs none
# (VTD_ENC_SPLITK=0): model / batch-parity tests, then forward A/B
set -o pipefail
O=gpurun_out/r6es
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_batch_parity.py tests/test_gpu_bf16x3.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "bf16x3 1" "bf16x3 8" "bf16x3 16" "bf16x3 32" "bf16 1" "bf16 8" "bf16 16" "bf16 32" "bf16 64" "bf16 256"; do
  set -- $cfg
  for es in 0 1; do
    VTD_ENC_SPLITK=$es timeout -k 10 300 python bench.py --dtype $1 --batch $2 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 b=$2 enc_splitk=$es', d['value'], 'img/s', d['ms_per_step'], 'ms')" || exit 1
  done
done
