"""Per-launch HBM traffic of the GEMM kernels from rocprofv3 PMC passes of bench.py.

FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (they cannot share one).
Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reports half the bytes of a wide coalesced
streaming read on gfx950 (16 B/lane, global_load and LDS-DMA alike), so it is doubled.
WRITE_SIZE is exact for 16-B-per-lane stores.  Both are in KiB.
  python tools/pmc_traffic.py <fetch_dir> <write_dir> [out.json]
"""
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter or "gemm_tn" not in r["Kernel_Name"]:
            continue
        key = r["Dispatch_Id"]
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return vals


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    nf, nw = len(fetch), len(write)
    fb = 2 * 1024 * sum(fetch.values()) / max(1, nf)
    wb = 1024 * sum(write.values()) / max(1, nw)
    out = {"kernel": "gemm_tn_* (all Dense layers)", "launches_fetch_pass": nf,
           "launches_write_pass": nw, "fetch_bytes_per_launch": fb,
           "write_bytes_per_launch": wb, "traffic_bytes_per_launch": fb + wb,
           "correction": "FETCH_SIZE x 2 (gfx950 wide-read undercount), WRITE_SIZE x 1; KiB"}
    if len(sys.argv) > 3:
        out["source"] = sys.argv[3]        # bench.py names it in roofline.traffic_source
        json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
