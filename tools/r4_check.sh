# Round-4 check: the new tests first, then the whole -m gpu suite, then the baseline
# measurements (tools/r4_baseline.sh).   gpurun --timeout 1200 -- bash tools/r4_check.sh
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_model.py -k "single_layer_mlp or concurrent_split" tests/test_gpu_kernels.py::test_gemm_statout_needs_a_specialised_epilogue > gpurun_out/r4b/new_tests.log 2>&1 || { tail -40 gpurun_out/r4b/new_tests.log; exit 1; }
tail -3 gpurun_out/r4b/new_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4b/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4b/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4b/gpu_tests.log
bash tools/r4_baseline.sh
