"""One forward of a rocprofv3 kernel trace (bench.py, default two-stream run): span, time with
0 / 1 / 2+ kernels running, per-kernel totals, and the head section (from the last encoder
GEMM to the end).  Forwards are delimited by the patch kernels (one per micro-batch).
  python tools/trace_forward2.py <kernel_trace.csv> [k (forward index, default 8)] [parts (2)]
"""
import collections
import csv
import re
import sys


def short(n):
    m = re.search(r"vtd::\(anonymous namespace\)::(\w+)(<[^>(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


def main(path, k=8, parts=2):
    rows = [r for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    pat = [i for i, r in enumerate(rows) if "patches" in r["Kernel_Name"]]
    s, e = pat[parts * k], pat[parts * (k + 1)]
    fw = rows[s:e]
    t0 = int(fw[0]["Start_Timestamp"])
    tend = max(int(r["End_Timestamp"]) for r in fw)
    ev = sorted([(int(r["Start_Timestamp"]), 1) for r in fw] + [(int(r["End_Timestamp"]), -1) for r in fw])
    cur, last, acc = 0, t0, collections.Counter()
    for t, d in ev:
        acc[min(cur, 2)] += t - last
        cur += d
        last = t
    print(f"span {(tend - t0) / 1e3:.1f} us; running kernels: " +
          ", ".join(f"{c}{'+' if c == 2 else ''}: {v / 1e3:.1f} us" for c, v in sorted(acc.items())))
    tot, cnt = collections.Counter(), collections.Counter()
    for r in fw:
        n = short(r["Kernel_Name"])
        tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[n] += 1
    for n, v in tot.most_common():
        print(f"{v:9.1f} {cnt[n]:4d} {v / cnt[n]:8.1f} {n}")
    # head: after the last residual GEMM of the encoder (the last pp2<13,...> launch)
    last_enc = max(i for i, r in enumerate(fw) if "pp2_kernel<13" in r["Kernel_Name"])
    h0 = int(fw[last_enc]["End_Timestamp"])
    print(f"\nhead section: {(tend - h0) / 1e3:.1f} us")
    for r in fw[last_enc - 1:]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} q{r['Queue_Id']} {short(r['Kernel_Name'])} "
              f"grid={r['Grid_Size_X']}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8,
         int(sys.argv[3]) if len(sys.argv) > 3 else 2)
