#!/bin/bash
# C2 forward with the streaming attention kernel (VTD_ATTN_VARIANT=2) vs the persistent one
# (default); C5 (ViT-L/16 @384, B = 128) fp8 / bf16 lines at the current build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/c5; mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local lab=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 240 python bench.py --no-cpu-baseline --no-parity-mode "$@" > $O/$lab.log 2>&1 || { tail -5 $O/$lab.log; exit 1; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*\|"mfma_util_attn_mlp": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' ')"
}
for r in 1 2; do
  run c2_attn4_$r X=1 -- --steps 30 || exit 1
  run c2_attn2_$r VTD_ATTN_VARIANT=2 -- --steps 30 || exit 1
done
for r in 1 2; do
  run c5_fp8_$r X=1 -- --preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3 || exit 1
  run c5_bf16_$r X=1 -- --preset vit_l16_384 --batch 128 --dtype bf16 --steps 10 --warmup 3 || exit 1
done
grep -o '"kernels": {.*}, "profiled' $O/c5_fp8_1.log | head -c 900; echo
grep -o '"kernels": {.*}, "profiled' $O/c5_bf16_1.log | head -c 900; echo
echo done
