"""Per-dispatch timeline of one vtd_forward from a rocprofv3 --kernel-trace CSV: the last
complete forward (patches kernel .. decode kernel), each dispatch with its duration, grid
and the idle gap before it, plus per-role totals.  Usage: python tools/trace_forward.py CSV [k]
(k = which forward from the end, default 1)."""
import csv
import re
import sys


def short(name):
    m = re.search(r"vtd::\(anonymous namespace\)::(\w+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main(path, k=1):
    rows = [r for r in csv.DictReader(open(path)) if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "patches" in r["Kernel_Name"]]
    ends = [i for i, r in enumerate(rows) if "decode_kernel" in r["Kernel_Name"]]
    s = starts[-k]
    e = min(i for i in ends if i > s)
    fw = rows[s:e + 1]
    t0 = int(fw[0]["Start_Timestamp"])
    prev_end = t0
    tot = {}
    busy = 0
    for r in fw:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        nm = short(r["Kernel_Name"])
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} us gap {(st - prev_end) / 1e3:6.1f} "
              f"q{r['Queue_Id']} wg {grid:6d} {nm}")
        tot[nm] = tot.get(nm, 0) + (en - st)
        busy += en - st
        prev_end = max(prev_end, en)
    span = (prev_end - t0) / 1e3
    print(f"forward span {span:.1f} us, sum of kernel times {busy / 1e3:.1f} us")
    for nm, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {v / 1e3:9.1f} us  {nm}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
