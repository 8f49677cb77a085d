# 8-wave streaming attention as the long-sequence default: tests + C3 / C5 forwards vs knob 2-equivalent old default
set -o pipefail
mkdir -p gpurun_out/r6a8
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py tests/test_gpu_model.py tests/test_gpu_batch_parity.py -k "attention or c3 or c5 or seeded" > gpurun_out/r6a8/tests.log 2>&1 || { tail -30 gpurun_out/r6a8/tests.log; exit 1; }
tail -1 gpurun_out/r6a8/tests.log
for rnd in 1 2; do
  for cfg in "c3:--preset vit_b16_640 --batch 32" "c5:--preset vit_l16_384 --batch 128 --steps 10 --warmup 3"; do
    lab=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['value'], d['mfma_util_attn_mlp'], d['roofline']['step_frac'], d['kernels']['attention']['avg_us'])" || exit 1
  done
done
