"""Overlap summary of one split (multi-stream) forward in a rocprofv3 kernel trace: span,
time with 0/1/2+ kernels running, per-kernel totals.  Usage: trace_overlap.py CSV [k]
(k-th split forward, counting patches kernels in pairs from the start; default 4)."""
import csv
import re
import sys


def short(n):
    m = re.search(r"vtd::\(anonymous namespace\)::(\w+)(<[^>(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:30]


def main(path, k=4, show=40):
    rows = [r for r in csv.DictReader(open(path)) if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    pat = [i for i, r in enumerate(rows) if "patches" in r["Kernel_Name"]]
    dec = [i for i, r in enumerate(rows) if "decode_kernel" in r["Kernel_Name"]]
    s = pat[2 * k]
    e = [i for i in dec if i > s][1]
    fw = rows[s:e + 1]
    t0 = int(fw[0]["Start_Timestamp"])
    tend = max(int(r["End_Timestamp"]) for r in fw)
    ev = sorted([(int(r["Start_Timestamp"]), 1) for r in fw] + [(int(r["End_Timestamp"]), -1) for r in fw])
    cur, last, acc = 0, t0, {}
    for t, d in ev:
        acc[min(cur, 2)] = acc.get(min(cur, 2), 0) + t - last
        cur += d
        last = t
    print(f"span {(tend - t0) / 1e3:.1f} us; running kernels: " +
          ", ".join(f"{c}{'+' if c == 2 else ''}: {v / 1e3:.1f} us" for c, v in sorted(acc.items())))
    for r in fw[:show]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} q{r['Queue_Id']} {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
