"""Summarise a rocprofv3 --pmc run: mean counter value per dispatch, grouped by
(kernel, grid size), so several shapes of one kernel in one run stay apart.
  python tools/pmc_summary.py <rocprof_out_dir> [kernel_substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(float))   # (kernel, grid, dispatch) -> counter -> sum
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if flt not in k:
                continue
            key = (k[:60], r.get("Grid_Size", "?"), r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    groups = defaultdict(list)
    for (k, g, _), c in per.items():
        groups[(k, g)].append(c)
    for (k, g), lst in sorted(groups.items()):
        print(f"{k} grid={g} dispatches={len(lst)}")
        names = sorted(lst[0])
        for n in names:
            v = sum(x.get(n, 0.0) for x in lst[1:] or lst) / max(1, len(lst[1:] or lst))
            print(f"    {n:32s} {v:16.1f}")


if __name__ == "__main__":
    main()
