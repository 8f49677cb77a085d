"""Print per-kernel VGPR / scratch / occupancy from hipcc -Rpass-analysis output.
  python tools/kres.py path/to/file.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c",
                      src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
    if "occ" in cur and "name" in cur:
        if flt in cur["name"]:
            print(f"{cur.get('vgpr'):4} vgpr {cur.get('scratch'):4} scratch occ {cur['occ']}  {cur['name'][:90]}")
        cur = {}
