# K-loop synchronisation cost: diagnostic build, VTD_PP2_DG = 0 / 32 (no per-phase barriers,
# wrong outputs) / 8 (no epilogue) / 40 (both), per-shape timings; + a product-library test subset.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c13
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "256_tile_path or accumulator_layouts" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for dg in 0 32 8 40; do
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_diag.so VTD_PP2_DG=$dg timeout -k 10 120 python tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st --reps 20 > $O/dg_$dg.jsonl 2>&1 || { tail -5 $O/dg_$dg.jsonl; exit 1; }
  echo "dg=$dg $(python3 -c "import json; print(' '.join(f\"{j['shape']}={j['us']}\" for j in map(json.loads, (l for l in open('$O/dg_$dg.jsonl') if l.startswith('{')))))")"
done
