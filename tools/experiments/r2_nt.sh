# non-temporal GEMM output stores (build-time VTD_OUT_NT=1, libvtd_nt.so) vs default stores:
# isolated shapes and forward bench, interleaved on one box
set -o pipefail
P=vision_transformer_detector_amd
rm -f gpurun_out/r2_nt.jsonl
for rep in 1 2; do for l in libvtd.so libvtd_nt.so; do
  VTD_LIB_PATH=$P/$l timeout -k 10 200 python3 tools/gemm_bench.py --reps 10 --shapes qkv,attn_out,mlp1,mlp2,mlp3 2>/dev/null | sed "s/^/$l /" >> gpurun_out/r2_nt.jsonl || exit 1
done; done
cat gpurun_out/r2_nt.jsonl
for rep in 1 2 3; do for l in libvtd.so libvtd_nt.so; do
  VTD_LIB_PATH=$P/$l timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_nt_bench.log 2>&1 || { tail -5 gpurun_out/r2_nt_bench.log; exit 1; }
  echo "BENCH $l $(tail -1 gpurun_out/r2_nt_bench.log | grep -o '"value": [0-9.]*')"
done; done
