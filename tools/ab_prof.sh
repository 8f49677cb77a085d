# rocprofv3 kernel stats of the bench for two arms (gpurun -- bash tools/ab_prof.sh VAR=value)
set -o pipefail
R=$GRAFT_REPO_ROOT
AB="$1"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_a -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_a.log 2>&1 || { tail -20 $R/gpurun_out/prof_a.log; exit 1; }
export $AB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_b.log 2>&1 || { tail -20 $R/gpurun_out/prof_b.log; exit 1; }
python3 - $R <<'PY'
import csv, glob, sys
R = sys.argv[1]
for arm in "ab":
    f = glob.glob(f"{R}/gpurun_out/prof_{arm}/**/*kernel_stats.csv", recursive=True)[0]
    print("arm", arm)
    for r in list(csv.DictReader(open(f)))[:9]:
        n = r["Name"]
        n = n[n.find("::", 20) + 2:][:58] if "vtd" in n else n[:58]
        print(f'  {n:60s} {r["Calls"]:>5} {float(r["AverageNs"]) / 1e3:9.1f}us')
PY
