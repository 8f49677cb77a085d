#!/bin/bash
# Persistent attention at C2: average shader clock per mode (GRBM_GUI_ACTIVE / duration) and
# SQ busy counters, diag library modes 0 (full), 2 (DMAs + stores), 4 (compute + stores).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/attn_clk; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in 0 2 4; do
  VTD_LIB_PATH=$GRAFT_REPO_ROOT/vision_transformer_detector_amd/libvtd_diag.so VTD_ATTN_DMODE=$m \
    timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/m$m -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/attn_bench.py --reps 10 > $O/m$m.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for m in 0 2 4; do
  f=$(find $O/m$m -name '*counter_collection.csv' | head -1)
  python3 - "$f" $m <<'PY'
import csv, sys, collections
f, m = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); dur = {}
for r in csv.DictReader(open(f)):
    if 'attention' not in r['Kernel_Name']: continue
    d = r['Dispatch_Id']; acc[d][r['Counter_Name']] += float(r['Counter_Value'])
    dur[d] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) if 'End_Timestamp' in r else None
ks = sorted(acc, key=int)[3:]
avg = {c: sum(acc[d][c] for d in ks) / len(ks) for c in acc[ks[0]]}
us = sum(dur[d] for d in ks) / len(ks) / 1e3 if dur[ks[0]] else float('nan')
print(f"mode {m}: {len(ks)} dispatches, {us:.1f} us, GRBM_GUI_ACTIVE/XCD {avg['GRBM_GUI_ACTIVE']/8:.0f} -> {avg['GRBM_GUI_ACTIVE']/8/us/1e3:.2f} GHz, "
      + ", ".join(f"{c} {v:.3g}" for c, v in avg.items()))
PY
done
find $O -name '*.csv' -size +5M -delete
