"""Per-shape HBM traffic / L2 hit rate of the GEMM kernels from rocprofv3 PMC passes of
tools/gemm_bench.py (one pass per counter group; FETCH_SIZE and WRITE_SIZE cannot share one).

Launches are grouped by (kernel name, grid size); each group is matched to the
gemm_bench shape with that tile count.  FETCH_SIZE is doubled (gfx950 reports half the
bytes of a wide coalesced read, MI355X_MICROARCH.md §HBM), WRITE_SIZE taken as is; both
are KiB.  Algorithmic bytes per launch: A, Bt, the output and (residual layers) the
residual, each once.
  python tools/pmc_per_shape.py <fetch_dir> <write_dir> [<tcc_dir>] [out.json]
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_bench import SHAPES  # noqa: E402


def tiles(M, N):
    return ((M + 255) // 256) * ((N + 255) // 256)


def shape_of(kernel, grid):
    """gemm_bench shape of a pp2 launch: tile count + the epilogue code's residual and
    activation bits (kernel template argument)."""
    import re
    wg = grid // 512 if grid % 512 == 0 else grid
    m = re.search(r"pp2_kernel<(-?\d+)", kernel)
    code = int(m.group(1)) if m else -1
    resid, act = code >= 0 and bool(code & 8), code & 3 if code >= 0 else -1
    for name, (M, N, K, a, od, res) in SHAPES.items():
        if (tiles(M, N) == wg and res == resid and (a != 0) == (act != 0) and
                not name.endswith(("_noact", "_st", "_ln", "_h"))):
            return name
    return f"{kernel[:40]}|{wg}"


def collect(d, counters):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return {}
    per = {}
    for r in csv.DictReader(open(files[0])):
        if r["Counter_Name"] not in counters or "gemm" not in r["Kernel_Name"]:
            continue
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", "0")) or 0)
        key = (r["Kernel_Name"], grid)
        disp = per.setdefault(key, {})
        dd = disp.setdefault(r["Dispatch_Id"], {})
        dd[r["Counter_Name"]] = dd.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def main():
    fetch = collect(sys.argv[1], {"FETCH_SIZE"})
    write = collect(sys.argv[2], {"WRITE_SIZE"})
    tcc = collect(sys.argv[3], {"TCC_HIT_sum", "TCC_MISS_sum"}) if len(sys.argv) > 3 else {}
    rows = {}
    for (k, g), disp in fetch.items():
        s = shape_of(k, g)
        v = [x["FETCH_SIZE"] for x in disp.values()]
        rows.setdefault(s, {})["fetch_MB"] = round(2 * 1024 * sum(v) / len(v) / 1e6, 1)
        rows[s]["launches"] = len(v)
    for (k, g), disp in write.items():
        s = shape_of(k, g)
        v = [x["WRITE_SIZE"] for x in disp.values()]
        rows.setdefault(s, {})["write_MB"] = round(1024 * sum(v) / len(v) / 1e6, 1)
    for (k, g), disp in tcc.items():
        s = shape_of(k, g)
        h = sum(x.get("TCC_HIT_sum", 0) for x in disp.values())
        m = sum(x.get("TCC_MISS_sum", 0) for x in disp.values())
        rows.setdefault(s, {})["l2_hit"] = round(h / max(1.0, h + m), 3)
    for s, r in rows.items():
        if s in SHAPES:
            M, N, K, act, od, res = SHAPES[s]
            alg = 2 * (M * K + N * K + M * N * (2 if res else 1))
            r["alg_MB"] = round(alg / 1e6, 1)
            if "fetch_MB" in r and "write_MB" in r:
                r["traffic_over_alg"] = round((r["fetch_MB"] + r["write_MB"]) / r["alg_MB"], 2)
                r["fetch_over_operands"] = round(
                    r["fetch_MB"] / (2 * (M * K + N * K + (M * N if res else 0)) / 1e6), 2)
    out = {"correction": "FETCH_SIZE x 2, WRITE_SIZE x 1 (KiB -> MB)", "shapes": rows}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
