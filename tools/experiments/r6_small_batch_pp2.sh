# few-tile wide GEMMs on the 256-tile kernels (default now) vs the 128 x 128 register-staged kernel
# (VTD_SMALL_PP2=0): kernel / model tests, then forward A/B at small and large batches
set -o pipefail
O=gpurun_out/r6sp
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bf16x3.py tests/test_gpu_batch_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "bf16x3 1" "bf16x3 8" "bf16x3 32" "bf16 1" "bf16 8" "bf16 32" "bf16 64" "f32 8" "bf16 256" "bf16x3 256"; do
  set -- $cfg
  for sp in 0 1; do
    VTD_SMALL_PP2=$sp timeout -k 10 300 python bench.py --dtype $1 --batch $2 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 b=$2 small_pp2=$sp', d['value'], 'img/s', d['ms_per_step'], 'ms')" || exit 1
  done
done
