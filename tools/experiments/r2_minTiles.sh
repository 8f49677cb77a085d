# A/B of the 256-tile threshold (VTD_PP2_MIN_TILES) on the forward bench + model tests at 1
set -o pipefail
VTD_PP2_MIN_TILES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_batch_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r2_mt_tests.log 2>&1 || { tail -30 gpurun_out/r2_mt_tests.log; exit 1; }
tail -1 gpurun_out/r2_mt_tests.log
for t in 128 32 8 1 128 32 8 1; do
  VTD_PP2_MIN_TILES=$t timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_mt_bench_$t.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_mt_bench_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH min_tiles=$t', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'])"
done
