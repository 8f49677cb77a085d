# ping-pong long-sequence attention (knob 7) vs the streaming kernel (default): tests, kernel
# A/B at the C3 / C5 shapes, C3 / C5 forwards
set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py -k "attention" > gpurun_out/r6e/tests.log 2>&1 || { tail -30 gpurun_out/r6e/tests.log; exit 1; }
tail -2 gpurun_out/r6e/tests.log
timeout -k 10 100 python tools/attn_bench.py --B 32 --N 1600 --variants=-1,7 --reps 20 --rounds 3 2>/dev/null | grep dtype | tee gpurun_out/r6e/attn.log || exit 1
timeout -k 10 100 python tools/attn_bench.py --B 128 --N 576 --H 16 --variants=-1,7 --reps 20 --rounds 3 2>/dev/null | grep dtype | tee -a gpurun_out/r6e/attn.log || exit 1
for v in -1 7 -1 7; do
  VTD_ATTN_VARIANT=$v timeout -k 10 200 python bench.py --preset vit_b16_640 --batch 32 --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('v$v c3', d['value'], d['roofline']['step_frac'], d['kernels']['attention']['avg_us'])" | tee -a gpurun_out/r6e/bench.log || exit 1
done
