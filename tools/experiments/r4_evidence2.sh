# Round-4 evidence, part 2 (gpurun --timeout 1200 -- bash tools/r4_evidence2.sh <tag>): the other
# BASELINE configs' bench lines, per-shape GEMM timings against the vendor library, per-shape
# PMC traffic, and a one-forward kernel trace of the default two-stream run.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r4e2}
O=$R/gpurun_out/$T
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
  echo "$n $(tail -1 $O/bench_$n.log | cut -c1-200)"
}
run c2_b64_bf16 --batch 64
run c3_b32_bf16 --preset vit_b16_640 --batch 32
run c5_b128_fp8 --preset vit_l16_384 --batch 128 --dtype fp8
run c5_b128_bf16 --preset vit_l16_384 --batch 128
run c2_b256_f32 --dtype f32 --steps 5 --warmup 2
SH=qkv,qkv_ln,attn_out,attn_out_st,mlp1,mlp1_ln,mlp2,mlp3,mlp3_st,head1,head2,sq8192,mlp1_noact,mlp2_noact
VTD_GEMM_REF_LIB=1 timeout -k 10 240 python tools/gemm_bench.py --shapes $SH > $O/gemm_vs_vendor.jsonl 2>&1 || { tail -20 $O/gemm_vs_vendor.jsonl; exit 1; }
cut -c1-160 $O/gemm_vs_vendor.jsonl
cd /tmp && export TMPDIR=/tmp
PS=qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st,head1,head2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pw.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pt -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pt.log 2>&1 || exit 1
python3 $R/tools/pmc_per_shape.py $O/pf $O/pw $O/pt $O/traffic_per_shape.json > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_forward2.py $f 8 > $O/trace_summary.txt 2>&1 || true
head -3 $O/trace_summary.txt
echo done
