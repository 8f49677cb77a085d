#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python -u tools/r3_determinism.py 128 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_det.log
