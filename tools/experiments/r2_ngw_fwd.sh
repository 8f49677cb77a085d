# forward A/B: default tile order (n-groups of 4 / 3) vs row-major (VTD_GEMM_NGW=0)
set -o pipefail
for r in 1 2 3; do for g in 0 d; do
  if [ $g = d ]; then unset VTD_GEMM_NGW; else export VTD_GEMM_NGW=$g; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ngwf_$g.log 2>&1 || { tail -5 gpurun_out/ngwf_$g.log; exit 1; }
  echo "ngw $g $(tail -1 gpurun_out/ngwf_$g.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/ngwf_$g.log | grep -o '"frac": [0-9.]*')"
done; done
