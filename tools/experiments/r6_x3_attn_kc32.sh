# split-bf16 attention: 32-key chunks at two workgroups per CU (knob 9; 127 VGPRs, 72 KiB LDS)
# vs the default 64-key chunks at one (169 VGPRs, 84 KiB): tests, kernel A/B at C2 / C3, forward A/B
set -o pipefail
O=gpurun_out/r6kc
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16x3.py -k "attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/attn_bench.py --dtype x3 --variants=-1,9 --rounds 3 --reps 20 | tee $O/c2.jsonl
timeout -k 10 300 python tools/attn_bench.py --dtype x3 --B 32 --N 1600 --variants=-1,9 --rounds 2 --reps 10 | tee $O/c3.jsonl
for rnd in 1 2 3; do
  for v in -1 9; do
    VTD_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --dtype bf16x3 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('knob $v', d['value'], d['ms_per_step'], d['kernels']['attention']['avg_us'])" || exit 1
  done
done
