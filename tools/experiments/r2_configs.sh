# full GPU suite, then the other BASELINE configs: C5 fp8 (tile order default vs row-major),
# C2 B=64, C3 B=32
set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for r in 1 2; do for g in 0 d; do
  if [ $g = d ]; then unset VTD_GEMM_NGW; else export VTD_GEMM_NGW=$g; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 > gpurun_out/c5_$g.log 2>&1 || { tail -5 gpurun_out/c5_$g.log; exit 1; }
  echo "C5 fp8 ngw $g $(tail -1 gpurun_out/c5_$g.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/c5_$g.log | grep -o '"frac": [0-9.]*')"
done; done
unset VTD_GEMM_NGW
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 64 > gpurun_out/c2_b64.log 2>&1 || { tail -5 gpurun_out/c2_b64.log; exit 1; }
echo "C2 B64 $(tail -1 gpurun_out/c2_b64.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/c2_b64.log | grep -o '"frac": [0-9.]*')"
timeout -k 10 300 python bench.py --no-cpu-baseline --preset vit_b16_640 --batch 32 --steps 10 --warmup 3 > gpurun_out/c3_b32.log 2>&1 || { tail -5 gpurun_out/c3_b32.log; exit 1; }
echo "C3 B32 $(tail -1 gpurun_out/c3_b32.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/c3_b32.log | grep -o '"frac": [0-9.]*')"
