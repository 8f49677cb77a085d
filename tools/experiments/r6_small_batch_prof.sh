# where a small-batch forward spends its time: rocprofv3 kernel stats at B = 8 (bf16x3, bf16), one stream
set -o pipefail
O=gpurun_out/r6sbp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for dt in bf16x3 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$dt -o run --output-format csv -- python3 bench.py --dtype $dt --batch 8 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-mode > $O/$dt.log 2>&1 || exit 1
  python3 - $O/$dt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:14]:
    print(f"{int(r['Calls']):6d} {float(r['AverageNs'])/1000:9.1f} us {float(r['TotalDurationNs'])/1e6:9.2f} ms  {r['Name'][:110]}")
PY
done
