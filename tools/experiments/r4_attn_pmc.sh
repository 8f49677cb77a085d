# SQ counter passes over the attention kernels (C2 persistent 32- / 16-query, C3 streaming):
#   gpurun -- bash tools/r4_attn_pmc.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4attn
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_COUNT"
for i in 1 2; do
  eval P=\$P$i
  for cfg in "--variants 4 --N 196 --B 256" "--variants 5 --N 196 --B 256" "--variants -1 --N 1600 --B 32"; do
    tag=$(echo $cfg | tr -d ' -' )
    timeout -s KILL 90 rocprofv3 --pmc $P -d $O/p${i}_$tag -o p --output-format csv -- python3 $R/tools/attn_bench.py $cfg --reps 5 > $O/p${i}_$tag.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import csv, glob, os, collections
O = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/r4attn"
for d in sorted(glob.glob(O + "/p*")):
    if not os.path.isdir(d): continue
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f: continue
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if "attention" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(os.path.basename(d), {k: round(v / max(1, n[k]), 0) for k, v in acc.items()})
PY
echo done
