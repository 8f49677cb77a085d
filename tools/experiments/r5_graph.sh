#!/bin/bash
# Host-enqueue test: eager vtd_forward calls against one HIP-graph replay per step (bench
# --graph 1), C2 at B = 64 (one stream; two padded parts) and B = 256, interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/graph; mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local lab=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 "$@" > $O/$lab.log 2>&1 || { tail -5 $O/$lab.log; exit 1; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*\|"mfma_util_attn_mlp": [0-9.]*' | tr '\n' ' ')"
}
for r in 1 2; do
  run b64_one_eager_$r X=1 -- --batch 64 || exit 1
  run b64_one_graph_$r X=1 -- --batch 64 --graph 1 || exit 1
  run b64_pad_eager_$r VTD_SPLIT_MIN_TILES=24 -- --batch 64 || exit 1
  run b64_pad_graph_$r VTD_SPLIT_MIN_TILES=24 -- --batch 64 --graph 1 || exit 1
  run b256_eager_$r X=1 -- --batch 256 || exit 1
  run b256_graph_$r X=1 -- --batch 256 --graph 1 || exit 1
done
echo done
