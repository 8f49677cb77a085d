# PNG decode tests + the JPEG / preprocessing tests (decode_images shares their buffers).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c11
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_png.py tests/test_gpu_jpeg.py tests/test_png_host.py tests/test_jpeg_host.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
