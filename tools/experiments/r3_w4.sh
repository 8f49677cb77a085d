#!/bin/bash
# round 3: w4 GEMM correctness + per-shape timing (w4 schedules 1 / 2, pp2, vendor), diagnostics
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
O=gpurun_out/r3_w4_bench5.jsonl
VTD_W4_SCHED=2 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "gemm" > gpurun_out/r3_w4_tests5.log 2>&1 || { tail -30 gpurun_out/r3_w4_tests5.log; exit 1; }
tail -2 gpurun_out/r3_w4_tests5.log
SH=qkv,attn_out,mlp1,mlp2,mlp3,head2,sq8192
VTD_GEMM_REF_LIB=1 timeout -k 10 200 python -u tools/gemm_bench.py --reps 20 --shapes $SH | sed 's/"variant": "default"/"variant": "w4s1"/' >> $O || exit 1
VTD_W4_SCHED=2 timeout -k 10 200 python -u tools/gemm_bench.py --reps 20 --shapes $SH | sed 's/"variant": "default"/"variant": "w4s2"/' >> $O || exit 1
VTD_GEMM_VARIANT=10 timeout -k 10 200 python -u tools/gemm_bench.py --reps 20 --shapes $SH >> $O || exit 1
for d in 1 2 3 4; do
  VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_diag.so VTD_W4_DG=$d timeout -k 10 200 python -u tools/gemm_bench.py --reps 20 --shapes qkv,sq8192 | sed "s/\"variant\": \"default\"/\"variant\": \"diag$d\"/" >> $O || exit 1
done
cat $O
