# bf16x3 (split-bf16 parity mode) forward: bench line (two streams) + one-stream kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6x3
mkdir -p $O
timeout -k 10 300 python bench.py --dtype bf16x3 --no-cpu-baseline --no-parity-mode > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 $R/bench.py --dtype bf16x3 --steps 5 --warmup 2 --no-cpu-baseline --no-parity-mode --streams 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["TotalDurationNs"])/tot*100:5.1f}% {float(r["AverageNs"])/1e3:8.1f}us x{r["Calls"]:>5} {r["Name"][:110]}')
PY
find $O -name '*kernel_trace.csv' -delete
