# after the compile-time wrap (PP2Src<AW>: the bf16 forward's pp2 codes issue without the
# wrap arithmetic): split-bf16 tests, then bf16 A/B vs libvtd_exp.so (-DVTD_NO_AWRAP build of
# the runtime-wrap source) and two bf16x3 lines
set -o pipefail
O=gpurun_out/r6x2b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bf16x3.py tests/test_gpu_model.py tests/test_gpu_kernels.py \
  -k "split or bf16x3 or splitk or gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rnd in 1 2 3; do
  for lib in prod exp; do
    if [ $lib = exp ]; then export VTD_LIB_PATH=$PWD/vision_transformer_detector_amd/libvtd_exp.so; else unset VTD_LIB_PATH; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'])" || exit 1
  done
done
unset VTD_LIB_PATH
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype bf16x3 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16x3', d['value'], d['ms_per_step'])" || exit 1
done
