# bf16 streaming attention with 32-key chunks (knob 11: 4-wave workgroups x 5 per CU, 96 VGPRs;
# 12: x 6, 80 VGPRs + spills; 13: 8-wave x 2, 101 VGPRs) vs the default (4: 8-wave 64-key, 126 VGPRs)
set -o pipefail
O=gpurun_out/r6kcb
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "test_attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/attn_bench.py --B 32 --N 1600 --variants=4,11,12,13 --rounds 3 --reps 10 | tee $O/c3.jsonl
timeout -k 10 300 python tools/attn_bench.py --B 128 --N 576 --H 16 --variants=4,11,12,13 --rounds 3 --reps 10 | tee $O/c5.jsonl
