# C2 B=64: micro-batch parts 2 (default) vs 3 / 4 (VTD_STREAMS, VTD_SPLIT_MIN_TILES), interleaved
set -o pipefail
for rnd in 1 2; do
  for cfg in "2:24" "3:16" "4:12"; do
    ns=${cfg%%:*}; mt=${cfg#*:}
    VTD_SPLIT_MIN_TILES=$mt timeout -k 10 200 python bench.py --batch 64 --streams $ns --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('parts=$ns', d['value'], d['mfma_util_attn_mlp'], d['roofline']['step_frac'])" || exit 1
  done
done
