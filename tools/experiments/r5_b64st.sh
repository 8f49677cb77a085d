#!/bin/bash
# New defaults (two padded parts from 24 tiles per part, 256-tile kernels from 64 tiles):
# full GPU suite, then C2 at B = 64 / 96 / 128 with stagger 0 / 1 / 2, and B = 256; interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/b64st; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  local lab=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 "$@" > $O/$lab.log 2>&1 || { tail -5 $O/$lab.log; exit 1; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*\|"mfma_util_attn_mlp": [0-9.]*' | tr '\n' ' ')"
}
for r in 1 2; do
  for b in 64 96 128; do
    for s in 0 1 2; do
      run b${b}_st${s}_$r VTD_STAGGER=$s -- --batch $b || exit 1
    done
    run b${b}_one_$r X=1 -- --batch $b --streams 1 || exit 1
  done
  run b256_$r X=1 -- --batch 256 || exit 1
done
echo done
