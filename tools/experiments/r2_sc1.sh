# sc1 (L2-dropping) GEMM output stores: tests under VTD_STORE_SC1=1, isolated shapes, L2 hit
# rate, forward bench A/B (0 / 1 interleaved)
set -o pipefail
R=$GRAFT_REPO_ROOT
VTD_STORE_SC1=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_batch_parity.py -m gpu -q -x -k "gemm or c2" --timeout 200 --timeout-method thread > gpurun_out/r2_sc1_tests.log 2>&1 || { tail -30 gpurun_out/r2_sc1_tests.log; exit 1; }
tail -1 gpurun_out/r2_sc1_tests.log
for v in 0 1 0 1; do
  VTD_STORE_SC1=$v timeout -k 10 200 python3 tools/gemm_bench.py --reps 10 --shapes qkv,attn_out,mlp1,mlp2,mlp3 2>/dev/null | sed "s/^/sc1=$v /" >> gpurun_out/r2_sc1.jsonl || exit 1
done
cat gpurun_out/r2_sc1.jsonl
cd /tmp && export TMPDIR=/tmp
VTD_STORE_SC1=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/l2hit_sc1 -o p --output-format csv -- python3 $R/tools/gemm_bench.py --reps 2 --shapes qkv,mlp1,mlp2 > /dev/null 2>&1 || exit 1
cd $R
for v in 0 1 0 1; do
  VTD_STORE_SC1=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2_sc1_bench_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/r2_sc1_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH sc1=$v', d['value'], d['mfma_util_attn_mlp'], d['roofline']['frac'])"
done
