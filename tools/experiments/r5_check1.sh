#!/bin/bash
# round 5: first GPU pass of the split-bf16 mode (kernel tests, goldens, bench with parity_mode)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5c1
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_bf16x3.py tests/test_gpu_png.py > gpurun_out/r5c1/t1.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_model.py tests/test_gpu_batch_parity.py -k "bf16x3" > gpurun_out/r5c1/t2.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5c1/bench.log 2>&1
rc=$?
tail -5 gpurun_out/r5c1/*.log
exit $rc
