#!/bin/bash
# asm_peek.sh <file.hip> <kernel-substring>: compile for gfx950, print the kernel's
# s_waitcnt / vmem / barrier / branch skeleton (for checking counted waits by eye)
set -e
f=$(realpath $1); k=$2
d=$(mktemp -d)
( cd $d && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast \
    -c $f --save-temps -o x.o 2>/dev/null )
python3 - "$d" "$k" <<'PY'
import sys, glob
d, k = sys.argv[1], sys.argv[2]
s = open(glob.glob(d + "/*gfx950*.s")[0]).read()
names = [l.split(':')[0] for l in s.splitlines() if ':' in l and k in l.split(':')[0] and not l.startswith(('.', ' ', '\t'))]
name = names[0]
i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
body = s[i:j].splitlines()
open('/tmp/peek.s', 'w').write('\n'.join(body))
for n, l in enumerate(body):
    t = l.strip()
    if any(x in t for x in ('waitcnt', 'buffer_', 'global_', 's_barrier', 's_cbranch', 'ds_read', 'ds_write')) or t.startswith('.LBB'):
        print(n, t)
PY
rm -rf $d
