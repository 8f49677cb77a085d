#!/bin/bash
# Head split-K workgroup target per launch (VTD_SPLITK: 0 = no split-K, >= 64 = the target;
# default 256) with the two micro-batch halves' head launches co-running; C2 B = 256 and 64.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/splitk; mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local lab=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 "$@" > $O/$lab.log 2>&1 || { tail -5 $O/$lab.log; exit 1; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*\|"mfma_util_attn_mlp": [0-9.]*' | tr '\n' ' ')"
}
for r in 1 2; do
  for k in -1 128 96 64 0; do
    run b256_sk${k}_$r VTD_SPLITK=$k -- --batch 256 || exit 1
  done
  for k in -1 128 0; do
    run b64_sk${k}_$r VTD_SPLITK=$k -- --batch 64 || exit 1
  done
done
echo done
