#!/bin/bash
# Kernel trace of C2 at B = 64 with the round-5 defaults (two padded parts, stagger 1)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace64b; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/split -o p --output-format csv -- python3 $R/bench.py --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode > $O/split.log 2>&1 || { tail -20 $O/split.log; exit 1; }
cd $R
f=$(find $O/split -name '*kernel_trace.csv' | head -1)
python3 tools/trace_forward2.py $f 8 2 > $O/split.summary.txt 2>&1 || true
cat $O/split.summary.txt
python3 - $f <<'PY'
import csv, sys, re
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pat = [i for i, r in enumerate(rows) if "patches" in r["Kernel_Name"]]
s, e = pat[16], pat[18]
fw = rows[s:e]
t0 = int(fw[0]["Start_Timestamp"])
for r in fw[:80]:
    m = re.search(r"vtd::\(anonymous namespace\)::(\w+)(<[^>(]*>)?", r["Kernel_Name"])
    n = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} q{r['Queue_Id']} {n} grid={r['Grid_Size_X']}")
PY
rm -f $f
