"""Evidence hygiene: keep at the top of profiles/ only the files DESIGN.md / BASELINE.md /
README.md / INTEGRATION.md (and bench.py) cite; move every other file into profiles/archive/.
Citations are file names (with or without the profiles/ prefix), brace sets
(`r05_s7_rocprof_kernel_stats_{streams1,default}.csv`) and `.. ` ranges of numbered passes
(`r02_gemm_traffic_s2.json` .. `_s4.json`).
  python tools/profiles_prune.py [--dry-run]"""
import itertools
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
DOCS = ["DESIGN.md", "BASELINE.md", "README.md", "INTEGRATION.md", "bench.py"]
TOK = re.compile(r"(?:profiles/)?((?:r\d\d|gemm)_[A-Za-z0-9_.{},*\-]*[A-Za-z0-9}*])")


def expand(tok):
    parts = re.split(r"(\{[^}]*\})", tok)
    opts = [p[1:-1].split(",") if p.startswith("{") else [p] for p in parts]
    return {"".join(c) for c in itertools.product(*opts)}


def cited():
    names = set()
    for d in DOCS:
        text = open(os.path.join(ROOT, d)).read()
        for m in TOK.finditer(text):
            names |= expand(m.group(1))
        # numbered ranges: `X_s2.json` .. `_s4.json` -> X_s2 .. X_s4
        for m in re.finditer(r"(r\d\d_[A-Za-z0-9_]*?)_s(\d+)(\.[a-z]+)`?\s*\.\.\s*`?_s(\d+)", text):
            for k in range(int(m.group(2)), int(m.group(4)) + 1):
                names.add(f"{m.group(1)}_s{k}{m.group(3)}")
    return names


def main():
    dry = "--dry-run" in sys.argv
    import fnmatch
    keep = cited()
    pats = [n for n in keep if "*" in n]                    # `r06_s2_*`: every file it matches
    files = sorted(f for f in os.listdir(PROF) if os.path.isfile(os.path.join(PROF, f)))
    moved = [f for f in files if f not in keep and not any(fnmatch.fnmatch(f, p) for p in pats)]
    missing = sorted(n for n in keep if "." in n and "*" not in n and not os.path.exists(os.path.join(PROF, n))
                     and not os.path.exists(os.path.join(ROOT, n)))
    print(f"{len(files)} files, {len(files) - len(moved)} cited, {len(moved)} to archive/")
    for n in missing:
        print("cited but absent:", n)
    if dry:
        return
    os.makedirs(os.path.join(PROF, "archive"), exist_ok=True)
    for f in moved:
        shutil.move(os.path.join(PROF, f), os.path.join(PROF, "archive", f))


if __name__ == "__main__":
    main()
