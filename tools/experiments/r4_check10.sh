# Head split-K workgroup target A/B (VTD_SPLITK = default 256 / 384 / 512 / 768), forward, 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c10
mkdir -p $O
for r in 1 2; do
  for v in -1 384 512 768; do
    VTD_SPLITK=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/b_${v}_$r.log 2>&1 || { tail -5 $O/b_${v}_$r.log; exit 1; }
    echo "splitk=$v r$r $(tail -1 $O/b_${v}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
