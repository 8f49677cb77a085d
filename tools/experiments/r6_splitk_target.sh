# head split-K workgroup target (VTD_SPLITK >= 64; default 256 / concurrent parts = 128 at C2 B=256,
# which leaves head2's 153 tiles per part unsplit): 256 / 384 / 512 split head2 2 / 3 / 4 ways
set -o pipefail
for rnd in 1 2 3; do
  for t in -1 256 384 512; do
    if [ $t = -1 ]; then unset VTD_SPLITK; else export VTD_SPLITK=$t; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('target $t', d['value'], d['ms_per_step'])" || exit 1
  done
done
