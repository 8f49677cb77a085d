set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > gpurun_out/r4ab_tests.log 2>&1 || { tail -30 gpurun_out/r4ab_tests.log; exit 1; }
tail -1 gpurun_out/r4ab_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_batch_parity.py tests/test_gpu_model.py > gpurun_out/r4ab_tests2.log 2>&1 || { tail -30 gpurun_out/r4ab_tests2.log; exit 1; }
tail -1 gpurun_out/r4ab_tests2.log
bash tools/r4_ab.sh vision_transformer_detector_amd/libvtd_base.so vision_transformer_detector_amd/libvtd.so 3
