# tile-order A/B, second pass: qkv / mlp1 / mlp2 / head1 at more reps, g = 0, 2, 3, 4
set -o pipefail
rm -f gpurun_out/ngw_micro2.jsonl
for r in 1 2 3; do for g in 0 2 3 4; do
  VTD_GEMM_NGW=$g timeout -k 10 200 python3 tools/gemm_bench.py --reps 20 --shapes qkv,mlp1,mlp2,head1 > gpurun_out/ngw_one.jsonl 2>/dev/null || exit 1
  sed "s/^{/{\"ngw\": $g, /" gpurun_out/ngw_one.jsonl >> gpurun_out/ngw_micro2.jsonl
done; done
python3 - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/ngw_micro2.jsonl"):
    r=json.loads(l); d[(r["shape"],r["ngw"])].append(r["us"])
for k in sorted(d): print(k, d[k], round(sum(d[k])/len(d[k]),1))
PY
