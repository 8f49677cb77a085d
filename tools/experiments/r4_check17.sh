# Skinny GEMM with the Bt staging loads batched: skinny / GEMM kernel tests, then per-shape
# timings of the head's skinny layers, interleaved against the previous build (libvtd_prev.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c17
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
S=det17,head272,head136,head6
for r in 1 2 3; do
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_prev.so timeout -k 10 120 python tools/gemm_bench.py --shapes $S --reps 50 > $O/gp_$r.jsonl 2>&1 || exit 1
  timeout -k 10 120 python tools/gemm_bench.py --shapes $S --reps 50 > $O/gn_$r.jsonl 2>&1 || exit 1
  for f in gp_$r gn_$r; do echo "$f $(python3 -c "import json; print(' '.join(f\"{j['shape']}={j['us']}\" for j in map(json.loads, (l for l in open('$O/$f.jsonl') if l.startswith('{')))))")"; done
done
for r in 1 2; do
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_prev.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/prev_$r.log 2>&1 || { tail -5 $O/prev_$r.log; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/new_$r.log 2>&1 || { tail -5 $O/new_$r.log; exit 1; }
  echo "r$r prev $(tail -1 $O/prev_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/new_$r.log | grep -o '"value": [0-9.]*')"
done
