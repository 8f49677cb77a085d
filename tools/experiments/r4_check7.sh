# JPEG (CMYK / YCCK) tests, then the multi-tile GEMM check (tools/r4_check6.sh).
#   gpurun --timeout 900 -- bash tools/r4_check7.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c7
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_jpeg.py > $O/jpeg.log 2>&1 || { tail -30 $O/jpeg.log; exit 1; }
tail -1 $O/jpeg.log
bash tools/r4_check6.sh
bash tools/r4_ab.sh vision_transformer_detector_amd/libvtd_prev.so vision_transformer_detector_amd/libvtd.so 2
