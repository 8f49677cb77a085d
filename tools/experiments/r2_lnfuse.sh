# fused LayerNorm finalize (the consumer pp2 GEMM merges the producer's partials; VTD_LN_FUSE=1,
# default) vs the finalize kernel (0): full GPU suite, then forward A/B interleaved
set -o pipefail
VTD_LN_FUSE=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
grep "worst max-rel" gpurun_out/gpu_tests.log | head -3
for r in 1 2 3; do for g in 0 1; do
  VTD_LN_FUSE=$g timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/lnf_$g.log 2>&1 || { tail -5 gpurun_out/lnf_$g.log; exit 1; }
  echo "lnfuse $g $(tail -1 gpurun_out/lnf_$g.log | grep -o '"value": [0-9.]*')"
done; done
