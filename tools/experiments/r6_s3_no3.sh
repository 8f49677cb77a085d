# upper bound of a two-piece split-bf16 operand: bf16x3 forward with the GEMM epilogues' third
# piece not stored (libvtd_exp.so, -DVTD_S3_NO3: WRONG outputs, timing only) vs the product library
# (the -DVTD_S3_NO3 guard lived in vtd_gemm.hip store_s3 at b9092bc; the two-piece operand replaced it)
set -o pipefail
for rnd in 1 2; do
  for lib in prod exp; do
    if [ $lib = exp ]; then export VTD_LIB_PATH=$PWD/vision_transformer_detector_amd/libvtd_exp.so; else unset VTD_LIB_PATH; fi
    timeout -k 10 300 python bench.py --dtype bf16x3 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'])" || exit 1
  done
done
