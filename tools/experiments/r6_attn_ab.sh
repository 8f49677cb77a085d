set -o pipefail
mkdir -p gpurun_out/r6c
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py tests/test_gpu_model.py tests/test_gpu_batch_parity.py -k "attention or seeded or c3 or c5 or tiny" > gpurun_out/r6c/tests.log 2>&1 || { tail -30 gpurun_out/r6c/tests.log; exit 1; }
tail -2 gpurun_out/r6c/tests.log
for lib in prev new; do
  if [ $lib = prev ]; then export VTD_LIB_PATH=$PWD/vision_transformer_detector_amd/libvtd_prev.so; else unset VTD_LIB_PATH; fi
  timeout -k 10 100 python tools/attn_bench.py --B 32 --N 1600 --variants -1 --reps 20 --rounds 2 2>/dev/null | sed "s/^/$lib /" >> gpurun_out/r6c/attn.log || exit 1
  timeout -k 10 100 python tools/attn_bench.py --B 128 --N 576 --H 16 --variants -1 --reps 20 --rounds 2 2>/dev/null | sed "s/^/$lib /" >> gpurun_out/r6c/attn.log || exit 1
done
cat gpurun_out/r6c/attn.log
for lib in prev new prev new; do
  if [ $lib = prev ]; then export VTD_LIB_PATH=$PWD/vision_transformer_detector_amd/libvtd_prev.so; else unset VTD_LIB_PATH; fi
  timeout -k 10 200 python bench.py --preset vit_b16_640 --batch 32 --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib c3', d['value'], d['roofline']['step_frac'], d['kernels']['attention']['avg_us'])" | tee -a gpurun_out/r6c/bench.log || exit 1
done
