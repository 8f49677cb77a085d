# C5 fp8 after restoring <= 128 VGPRs in the 8-wave attention (MX-fp8 epilogue) kernel
set -o pipefail
mkdir -p gpurun_out/r6c5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py tests/test_gpu_model.py tests/test_gpu_batch_parity.py -k "attention or c5 or c3 or tiny" > gpurun_out/r6c5/tests.log 2>&1 || { tail -30 gpurun_out/r6c5/tests.log; exit 1; }
tail -1 gpurun_out/r6c5/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 > gpurun_out/r6c5/bench_fp8_$i.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r6c5/bench_fp8_$i.log')); print('c5 fp8', d['value'], {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})"
done
