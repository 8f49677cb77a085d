# forward A/B of the persistent attention grid: one workgroup per CU (256) vs half (128)
set -o pipefail
for r in 1 2 3; do for g in 256 128; do
  VTD_ATTN_GRID=$g timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/agrid_$g.log 2>&1 || { tail -5 gpurun_out/agrid_$g.log; exit 1; }
  echo "grid $g $(tail -1 gpurun_out/agrid_$g.log | grep -o '"value": [0-9.]*')"
done; done
