#!/bin/bash
# Micro-batch parts padded to whole 256-row tiles (VTD_SPLIT_PAD, default on): C2 at B = 64 in
# two parts (VTD_SPLIT_MIN_TILES=24; 32 images = 6272 rows -> 6400) against one stream, the
# unpadded split, and staggered parts; C2 at B = 256 in 3 / 4 padded parts against 2.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/padsplit; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "two_stream or concurrent" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # label, env..., then bench args after --
  local lab=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 30 "$@" > $O/$lab.log 2>&1 || { tail -5 $O/$lab.log; exit 1; }
  echo "$lab $(tail -1 $O/$lab.log | grep -o '"value": [0-9.]*\|"mfma_util_attn_mlp": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' ')"
}
for r in 1 2; do
  run b64_one_$r X=1 -- --batch 64 || exit 1
  run b64_pad_$r VTD_SPLIT_MIN_TILES=24 -- --batch 64 || exit 1
  run b64_nopad_$r VTD_SPLIT_MIN_TILES=24 VTD_SPLIT_PAD=0 -- --batch 64 || exit 1
  run b64_pad_st1_$r VTD_SPLIT_MIN_TILES=24 VTD_STAGGER=1 -- --batch 64 || exit 1
  run b64_pad_st3_$r VTD_SPLIT_MIN_TILES=24 VTD_STAGGER=3 -- --batch 64 || exit 1
  run b256_s2_$r X=1 -- --batch 256 || exit 1
  run b256_s3_$r X=1 -- --batch 256 --streams 3 || exit 1
  run b256_s4_$r X=1 -- --batch 256 --streams 4 || exit 1
done
echo done
