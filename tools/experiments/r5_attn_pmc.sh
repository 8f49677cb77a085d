#!/bin/bash
# Round-5 attention evidence: per configuration one kernel-trace pass
# (duration) and four PMC passes (SQ x2, FETCH_SIZE, WRITE_SIZE) over tools/attn_bench.py;
# summary -> gpurun_out/r5attn/r05_attn_pmc.json.
#   gpurun -- bash tools/experiments/r5_attn_pmc.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5attn
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_COUNT"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for cfg in "c2:--N 196 --B 256 --H 12" "c3:--N 1600 --B 32 --H 12" "c5:--N 576 --B 128 --H 16"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/t_$tag -o t --output-format csv -- python3 $R/tools/attn_bench.py $args --reps 5 > $O/t_$tag.log 2>&1 || exit 1
  for i in 1 2 3 4; do
    eval P=\$P$i
    timeout -s KILL 90 rocprofv3 --pmc $P -d $O/p${i}_$tag -o p --output-format csv -- python3 $R/tools/attn_bench.py $args --reps 5 > $O/p${i}_$tag.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import csv, glob, os, collections, json
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r5attn"
shapes = {"c2": (256, 196, 12), "c3": (32, 1600, 12), "c5": (128, 576, 16)}
res = {"note": "rocprofv3 over tools/attn_bench.py (bf16, dk 64, default kernel per shape); per-dispatch "
               "averages of the attention kernel; FETCH_SIZE x 2 (gfx950 16-B/lane read undercount, "
               "MI355X_MICROARCH.md HBM section), WRITE_SIZE x 1, both KiB -> bytes; SQ_WAVE_CYCLES etc. "
               "in quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES in cycles (guide constants table)", "data": {}}
for tag, (B, N, H) in shapes.items():
    d = {}
    f = glob.glob(f"{O}/t_{tag}/**/*kernel_stats.csv", recursive=True)
    for r in csv.DictReader(open(f[0])):
        if "attention" in r["Name"]:
            d["kernel"] = r["Name"][:80]
            d["avg_us"] = round(float(r["AverageNs"]) / 1e3, 2)
            d["calls"] = int(r["Calls"])
    for i in (1, 2, 3, 4):
        f = glob.glob(f"{O}/p{i}_{tag}/**/*counter_collection.csv", recursive=True)
        acc = collections.defaultdict(float); disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f[0])):
            if "attention" not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for k, v in acc.items():
            d[k] = v / max(1, len(disp[k]))
    alg = 2 * B * N * H * 64 * 4          # Q, K, V read once, O written once (bf16)
    d["algorithmic_bytes"] = alg
    if "FETCH_SIZE" in d:
        d["fetch_bytes"] = 2 * 1024 * d["FETCH_SIZE"]
    if "WRITE_SIZE" in d:
        d["write_bytes"] = 1024 * d["WRITE_SIZE"]
    if "fetch_bytes" in d and "write_bytes" in d:
        d["traffic_bytes"] = d["fetch_bytes"] + d["write_bytes"]
        d["traffic_over_algorithmic"] = round(d["traffic_bytes"] / alg, 3)
    if "avg_us" in d:
        d["algorithmic_GBps"] = round(alg / d["avg_us"] / 1e3, 1)
        d["frac_of_hbm_8TBps"] = round(alg / d["avg_us"] / 1e3 / 8000, 3)
        d["attn_tflops"] = round(4.0 * B * H * N * N * 64 / d["avg_us"] / 1e6, 1)
    if "SQ_INSTS_VALU" in d and "SQ_INSTS_MFMA" in d and d["SQ_INSTS_MFMA"]:
        d["valu_per_mfma"] = round(d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"], 2)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d and d["GRBM_GUI_ACTIVE"]:
        # busy cycles summed over the 1024 SIMDs vs the kernel's GPU-active cycles (summed over 8 XCDs)
        d["mfma_busy_frac"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (d["GRBM_GUI_ACTIVE"] / 8), 3)
    res["data"][tag] = d
json.dump(res, open(O + "/r05_attn_pmc.json", "w"), indent=1)
for t, d in res["data"].items():
    print(t, {k: d.get(k) for k in ("avg_us", "algorithmic_GBps", "traffic_over_algorithmic", "valu_per_mfma", "mfma_busy_frac", "attn_tflops")})
PY
echo done
