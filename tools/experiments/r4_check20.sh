# Sub-stage stagger (VTD_SUBSTAGGER=k: the second micro-batch k sub-stages -- patch embedding,
# attention block, MLP block, head -- behind the first; odd k pairs attention with MLP GEMMs):
# model / batch-parity tests with k = 1, then an interleaved forward A/B (default, k = 1, k = 3).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c20
mkdir -p $O
VTD_SUBSTAGGER=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_batch_parity.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/def_$r.log 2>&1 || { tail -5 $O/def_$r.log; exit 1; }
  VTD_SUBSTAGGER=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/s1_$r.log 2>&1 || { tail -5 $O/s1_$r.log; exit 1; }
  VTD_SUBSTAGGER=3 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/s3_$r.log 2>&1 || { tail -5 $O/s3_$r.log; exit 1; }
  echo "r$r default $(tail -1 $O/def_$r.log | grep -o '"value": [0-9.]*') sub1 $(tail -1 $O/s1_$r.log | grep -o '"value": [0-9.]*') sub3 $(tail -1 $O/s3_$r.log | grep -o '"value": [0-9.]*')"
done
