# C2 B=64: one stream (default below 2 x 48 row tiles) vs two streams (VTD_SPLIT_MIN_TILES=24)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c12
mkdir -p $O
for r in 1 2; do
  for v in 48 24 12; do
    VTD_SPLIT_MIN_TILES=$v timeout -k 10 200 python bench.py --no-cpu-baseline --batch 64 --steps 40 > $O/b_${v}_$r.log 2>&1 || { tail -5 $O/b_${v}_$r.log; exit 1; }
    echo "min_tiles=$v r$r $(tail -1 $O/b_${v}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
for v in 128 192; do
  VTD_SPLIT_MIN_TILES=24 timeout -k 10 200 python bench.py --no-cpu-baseline --batch $v --steps 20 > $O/bb_${v}.log 2>&1 || { tail -5 $O/bb_${v}.log; exit 1; }
  VTD_SPLIT_MIN_TILES=48 timeout -k 10 200 python bench.py --no-cpu-baseline --batch $v --steps 20 > $O/bd_${v}.log 2>&1 || { tail -5 $O/bd_${v}.log; exit 1; }
  echo "batch=$v min24 $(tail -1 $O/bb_${v}.log | grep -o '"value": [0-9.]*') min48 $(tail -1 $O/bd_${v}.log | grep -o '"value": [0-9.]*')"
done
