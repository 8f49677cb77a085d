# A/B of alternative builds (VTD_LIB_PATH): isolated GEMM shapes + forward bench, interleaved
set -o pipefail
P=vision_transformer_detector_amd
LIBS=${LIBS:-"libvtd.so libvtd_ant.so libvtd_bsc0.so"}
for rep in 1 2; do
  for l in $LIBS; do
    VTD_LIB_PATH=$P/$l timeout -k 10 200 python3 tools/gemm_bench.py --reps 10 --shapes ${SHAPES:-qkv,attn_out,mlp1,mlp2,mlp3} 2>/dev/null | sed "s/^/$l /" >> gpurun_out/r2_libab.jsonl || exit 1
  done
done
cat gpurun_out/r2_libab.jsonl
for rep in 1 2; do
  for l in $LIBS; do
    VTD_LIB_PATH=$P/$l timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_libab_bench.log 2>&1 || exit 1
    tail -1 gpurun_out/r2_libab_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $l', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'])"
  done
done
