#!/bin/bash
# Copy an evidence pass (tools/r6_final.sh <tag>) from gpurun_out/<tag>/ into profiles/r06_<name>_*:
#   bash tools/evidence_copy.sh r6s5 s5
set -e
O=gpurun_out/$1; P=profiles/r06_$2
cp $O/bench.log ${P}_bench.log
for f in $O/bench_*.log; do cp $f ${P}_$(basename $f); done
cp $O/gpu_tests.log ${P}_gpu_tests.log
[ -f $O/smoke.log ] && cp $O/smoke.log ${P}_smoke.log
cp $O/accuracy.log ${P}_accuracy.log
cp $O/attn_pmc.json ${P}_attn_pmc.json
cp $(find $O/prof -name '*kernel_stats.csv' | head -1) ${P}_rocprof_kernel_stats_streams1.csv
cp $(find $O/prof2 -name '*kernel_stats.csv' | head -1) ${P}_rocprof_kernel_stats_default.csv
cp $O/trace_summary.txt ${P}_forward_trace_summary.txt
cp $O/gemm_traffic_per_shape.json ${P}_gemm_traffic_per_shape.json
python3 - "$O" "$P" "$2" <<'PY'
import json, sys
o, p, tag = sys.argv[1:]
d = json.load(open(f"{o}/gemm_traffic.json"))
d["source"] = f"round 6 {tag} pass, {o}/gemm_traffic.json"
json.dump(d, open(f"{p}_gemm_traffic.json", "w"), indent=1)
d["source"] = (f"{p}_gemm_traffic.json, round 6 {tag} pass (bench.py --streams 1 --no-parity-mode, "
               "C2 B=256 bf16)")
json.dump(d, open("profiles/gemm_traffic_latest.json", "w"), indent=1)
PY
