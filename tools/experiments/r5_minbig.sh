#!/bin/bash
# 256-tile kernels below 128 tiles (VTD_MIN_BIG_TILES): C2 B = 64 in two padded parts
# (75-tile N = 768 layers per part) and one stream, C2 B = 256; interleaved rounds.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/minbig; mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local lab=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 "$@" > $O/$lab.log 2>&1 || { tail -5 $O/$lab.log; exit 1; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*\|"mfma_util_attn_mlp": [0-9.]*' | tr '\n' ' ')"
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "two_stream" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  run b64_one_$r X=1 -- --batch 64 || exit 1
  run b64_one_mb32_$r VTD_MIN_BIG_TILES=32 -- --batch 64 || exit 1
  run b64_pad_mb64_$r VTD_SPLIT_MIN_TILES=24 VTD_MIN_BIG_TILES=64 -- --batch 64 || exit 1
  run b64_pad_mb32_$r VTD_SPLIT_MIN_TILES=24 VTD_MIN_BIG_TILES=32 -- --batch 64 || exit 1
  run b64_pad_mb32_st1_$r VTD_SPLIT_MIN_TILES=24 VTD_MIN_BIG_TILES=32 VTD_STAGGER=1 -- --batch 64 || exit 1
  run b256_$r X=1 -- --batch 256 || exit 1
  run b256_mb32_$r VTD_MIN_BIG_TILES=32 -- --batch 256 || exit 1
done
echo done
