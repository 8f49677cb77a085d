# Kernel arguments fetched in one batch: GEMM / model tests, then an interleaved forward A/B against the
# previous build (libvtd_prev.so), 3 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c16
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py tests/test_gpu_model.py tests/test_gpu_batch_parity.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_prev.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/prev_$r.log 2>&1 || { tail -5 $O/prev_$r.log; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/new_$r.log 2>&1 || { tail -5 $O/new_$r.log; exit 1; }
  echo "r$r prev $(tail -1 $O/prev_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/new_$r.log | grep -o '"value": [0-9.]*')"
done
VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_prev.so timeout -k 10 120 python tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st --reps 20 > $O/gp.jsonl 2>&1 || exit 1
timeout -k 10 120 python tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st --reps 20 > $O/gn.jsonl 2>&1 || exit 1
for f in gp gn; do echo "$f $(python3 -c "import json; print(' '.join(f\"{j['shape']}={j['us']}\" for j in map(json.loads, (l for l in open('$O/$f.jsonl') if l.startswith('{')))))")"; done
