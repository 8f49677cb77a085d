# GEMM tile order A/B: n-grouped (VTD_GEMM_NGW = g) vs row-major (0): kernel tests with g = 3,
# per-shape micro-benchmark interleaved, forward bench
set -o pipefail
VTD_GEMM_NGW=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/ngw_tests.log 2>&1 || { tail -30 gpurun_out/ngw_tests.log; exit 1; }
tail -1 gpurun_out/ngw_tests.log
rm -f gpurun_out/ngw_micro.jsonl
for r in 1 2; do for g in 0 2 3 4 6; do
  VTD_GEMM_NGW=$g timeout -k 10 200 python3 tools/gemm_bench.py --reps 10 --shapes qkv,attn_out,mlp1,mlp2,mlp3,head2 > gpurun_out/ngw_one.jsonl 2>/dev/null || exit 1
  sed "s/^{/{\"ngw\": $g, /" gpurun_out/ngw_one.jsonl >> gpurun_out/ngw_micro.jsonl
done; done
python3 - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/ngw_micro.jsonl"):
    r=json.loads(l); d[(r["shape"],r["ngw"])].append(r["us"])
for k in sorted(d): print(k, d[k])
PY
for g in 0 3 0 3; do
  VTD_GEMM_NGW=$g timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ngw_bench.log 2>&1 || { tail -5 gpurun_out/ngw_bench.log; exit 1; }
  echo "ngw $g $(tail -1 gpurun_out/ngw_bench.log | grep -o '"value": [0-9.]*')"
done
