# bf16 headline A/B: the product library (pp2 DMA issue with the split-bf16 A wrap's scalar
# arithmetic) vs libvtd_exp.so built with -DVTD_NO_AWRAP (the wrap left out; bf16 never wraps)
set -o pipefail
for rnd in 1 2 3; do
  for lib in prod exp; do
    if [ $lib = exp ]; then export VTD_LIB_PATH=$PWD/vision_transformer_detector_amd/libvtd_exp.so; else unset VTD_LIB_PATH; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'])" || exit 1
  done
done
