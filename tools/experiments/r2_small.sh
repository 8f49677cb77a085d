# LDS-DMA ring small GEMM (default) vs register-staged (VTD_GEMM_SMALL=0): kernel + model tests,
# forward A/B at C2 B=256 and B=64
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_batch_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/small_tests.log 2>&1 || { tail -30 gpurun_out/small_tests.log; exit 1; }
tail -1 gpurun_out/small_tests.log
for r in 1 2; do for g in 0 1; do
  export VTD_GEMM_SMALL=$g
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/small_$g.log 2>&1 || { tail -5 gpurun_out/small_$g.log; exit 1; }
  echo "B256 small=$g $(tail -1 gpurun_out/small_$g.log | grep -o '"value": [0-9.]*')"
  timeout -k 10 300 python bench.py --no-cpu-baseline --batch 64 > gpurun_out/small64_$g.log 2>&1 || { tail -5 gpurun_out/small64_$g.log; exit 1; }
  echo "B64 small=$g $(tail -1 gpurun_out/small64_$g.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/small64_$g.log | grep -o '"frac": [0-9.]*')"
done; done
