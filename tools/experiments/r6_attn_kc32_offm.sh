# bf16 streaming attention, 8-wave workgroups with 32-key chunks AND the in-MFMA running max /
# ones-block row sum (knob 13, 120 VGPRs: the tricks fit the 8-wave budget once the chunk halves)
# vs the default (4: 8-wave, 64-key chunks, no tricks, 126 VGPRs)
set -o pipefail
O=gpurun_out/r6kco
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "test_attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/attn_bench.py --B 32 --N 1600 --variants=4,13 --rounds 4 --reps 10 | tee $O/c3.jsonl
timeout -k 10 300 python tools/attn_bench.py --B 128 --N 576 --H 16 --variants=4,13 --rounds 4 --reps 10 | tee $O/c5.jsonl
