# Round-4 check: the new tests first, then the whole -m gpu suite, then the baseline
# measurements (tools/r4_baseline.sh).   gpurun --timeout 1200 -- bash tools/r4_check.sh
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_model.py::test_single_layer_mlp_fold_full_tiles tests/test_gpu_model.py::test_concurrent_split_forwards_on_two_streams tests/test_gpu_kernels.py::test_gemm_statout_needs_a_specialised_epilogue > gpurun_out/r4b/new_tests.log 2>&1 || { tail -40 gpurun_out/r4b/new_tests.log; exit 1; }
tail -3 gpurun_out/r4b/new_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "attention or reshape_scatter or skinny or f32_256 or stagger" tests/test_gpu_model.py > gpurun_out/r4b/attn_tests.log 2>&1 || { tail -40 gpurun_out/r4b/attn_tests.log; exit 1; }
tail -1 gpurun_out/r4b/attn_tests.log
timeout -k 10 200 python tools/attn_bench.py --variants 4,5 --rounds 3 > gpurun_out/r4b/attn_ab.jsonl 2>&1 || { tail -20 gpurun_out/r4b/attn_ab.jsonl; exit 1; }
cat gpurun_out/r4b/attn_ab.jsonl
for r in 1 2; do for v in 4 5; do
  VTD_ATTN_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r4b/fwd_attn_v$v.log 2>&1 || { tail -5 gpurun_out/r4b/fwd_attn_v$v.log; exit 1; }
  echo "attn variant $v round $r: $(tail -1 gpurun_out/r4b/fwd_attn_v$v.log | cut -c1-120)"
done; done
for r in 1 2; do for v in 0 1 2; do
  VTD_STAGGER=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r4b/fwd_stagger_$v.log 2>&1 || { tail -5 gpurun_out/r4b/fwd_stagger_$v.log; exit 1; }
  echo "stagger $v round $r: $(tail -1 gpurun_out/r4b/fwd_stagger_$v.log | cut -c1-120)"
done; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4b/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4b/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4b/gpu_tests.log
bash tools/r4_baseline.sh
