#!/bin/bash
# round 3: progressive JPEG decode tests (bit-exact vs Pillow's libjpeg-turbo) then the
# round-end evidence pass
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_jpeg.py -m gpu > gpurun_out/r3_jpeg_tests.log 2>&1 || { tail -40 gpurun_out/r3_jpeg_tests.log; exit 1; }
tail -1 gpurun_out/r3_jpeg_tests.log
bash tools/gpu_round_end.sh
