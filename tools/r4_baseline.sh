# Round-4 baseline on the GPU box: headline bench, per-shape GEMM timings (+ vendor library),
# per-shape PMC passes (FETCH_SIZE / WRITE_SIZE / TCC hit) of tools/gemm_bench.py.
#   gpurun --timeout 900 -- bash tools/r4_baseline.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
SH=qkv,attn_out,mlp1,mlp2,mlp3,head1,head2,sq8192,mlp1_noact,mlp2_noact
VTD_GEMM_REF_LIB=1 timeout -k 10 200 python tools/gemm_bench.py --shapes $SH > $O/gemm.jsonl 2>&1 || { tail -20 $O/gemm.jsonl; exit 1; }
cat $O/gemm.jsonl
cd /tmp && export TMPDIR=/tmp
PS=qkv,attn_out,mlp1,mlp2,mlp3,head1,head2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pw.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pt -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pt.log 2>&1 || exit 1
python3 $R/tools/pmc_per_shape.py $O/pf $O/pw $O/pt $O/traffic_per_shape.json
echo done
