# The LayerNorm-folded query/key/value GEMM on transposed accumulators (VTD_FOLD_TR=1):
# tests with it, an interleaved forward A/B, one-stream kernel stats of each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c22
mkdir -p $O
VTD_FOLD_TR=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_batch_parity.py -k "fold or layernorm or model or batch or logits" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/def_$r.log 2>&1 || { tail -5 $O/def_$r.log; exit 1; }
  VTD_FOLD_TR=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/tr_$r.log 2>&1 || { tail -5 $O/tr_$r.log; exit 1; }
  echo "r$r default $(tail -1 $O/def_$r.log | grep -o '"value": [0-9.]*') fold_tr $(tail -1 $O/tr_$r.log | grep -o '"value": [0-9.]*')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_def -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 1 > $O/prof_def.log 2>&1 || { tail -20 $O/prof_def.log; exit 1; }
export VTD_FOLD_TR=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tr -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 1 > $O/prof_tr.log 2>&1 || { tail -20 $O/prof_tr.log; exit 1; }
for v in def tr; do f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); echo "$v: $(grep -E 'pp2_kernel<36' $f | awk -F'","' '{split($1,a,"<"); print substr(a[2],1,9), $2, $4}' | tr '\n' ';')"; done
