# 16-query streaming attention (knob 8: 8 waves, 9: 4 waves) vs the 32-query streaming kernel
set -o pipefail
mkdir -p gpurun_out/r6s16
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention" > gpurun_out/r6s16/tests.log 2>&1 || { tail -30 gpurun_out/r6s16/tests.log; exit 1; }
tail -1 gpurun_out/r6s16/tests.log
timeout -k 10 100 python tools/attn_bench.py --B 32 --N 1600 --variants=-1,8,9 --reps 20 --rounds 3 2>/dev/null | grep dtype | tee gpurun_out/r6s16/attn.log || exit 1
timeout -k 10 100 python tools/attn_bench.py --B 128 --N 576 --H 16 --variants=-1,8,9 --reps 20 --rounds 2 2>/dev/null | grep dtype | tee -a gpurun_out/r6s16/attn.log || exit 1
timeout -k 10 100 python tools/attn_bench.py --B 256 --N 196 --variants=-1,8 --reps 20 --rounds 2 2>/dev/null | grep dtype | tee -a gpurun_out/r6s16/attn.log || exit 1
