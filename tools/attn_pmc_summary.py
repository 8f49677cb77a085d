"""Summary of the C3 attention passes of tools/r6_final.sh: kernel-trace duration and the SQ
counters of the attention kernel (per-dispatch averages) -> <dir>/attn_pmc.json.
  python tools/attn_pmc_summary.py gpurun_out/<tag>"""
import collections
import csv
import glob
import json
import sys

O = sys.argv[1]
B, N, H = 32, 1600, 12
d = {}
f = glob.glob(f"{O}/attn_t/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "attention" in r["Name"]:
        d["kernel"] = r["Name"][:80]
        d["avg_us"] = round(float(r["AverageNs"]) / 1e3, 2)
        d["calls"] = int(r["Calls"])
for i in (1, 2):
    f = glob.glob(f"{O}/attn_p{i}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        if "attention" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    for k, v in acc.items():
        d[k] = v / max(1, len(disp[k]))
if "avg_us" in d:
    d["attn_tflops"] = round(4.0 * B * H * N * N * 64 / d["avg_us"] / 1e6, 1)
    d["frac_of_bf16_peak"] = round(d["attn_tflops"] / 2516.6, 3)
if d.get("SQ_INSTS_MFMA"):
    # SQ_INSTS_VALU counts the MFMA instructions too: VALU per MFMA excluding them
    d["valu_per_mfma"] = round((d["SQ_INSTS_VALU"] - d["SQ_INSTS_MFMA"]) / d["SQ_INSTS_MFMA"], 2)
    d["valu_incl_mfma_per_mfma"] = round(d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"], 2)
if d.get("GRBM_GUI_ACTIVE"):
    d["mfma_busy_frac"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (d["GRBM_GUI_ACTIVE"] / 8), 3)
res = {"note": "rocprofv3 over tools/attn_bench.py --N 1600 --B 32 --H 12 (C3, bf16, default "
               "kernel); per-dispatch averages of the attention kernel; SQ_VALU_MFMA_BUSY_CYCLES "
               "in cycles summed over 1024 SIMDs, GRBM_GUI_ACTIVE summed over 8 XCDs",
       "c3": d}
json.dump(res, open(f"{O}/attn_pmc.json", "w"), indent=1)
print(json.dumps({k: d.get(k) for k in ("avg_us", "attn_tflops", "frac_of_bf16_peak",
                                         "valu_per_mfma", "valu_incl_mfma_per_mfma",
                                         "mfma_busy_frac")}))
