# two 32-query blocks per wave in the streaming bf16 attention (knob 7: 4-wave workgroups,
# 8: 8-wave) against the default 8-wave one-block kernel (4) at C3 / C5 shapes; correctness first
set -o pipefail
O=gpurun_out/r6qb
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "test_attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/attn_bench.py --B 32 --N 1600 --variants=4,7,8 --rounds 3 --reps 20 | tee $O/c3.jsonl
timeout -k 10 300 python tools/attn_bench.py --B 128 --N 576 --H 16 --variants=4,7,8 --rounds 3 --reps 20 | tee $O/c5.jsonl
