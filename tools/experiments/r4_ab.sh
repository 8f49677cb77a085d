# Interleaved A/B of two builds in one GPU call (VTD_LIB_PATH): per-shape GEMM timings and the
# headline bench, R rounds.   gpurun -- bash tools/r4_ab.sh <libA> <libB> [rounds] [shapes]
set -o pipefail
R=$GRAFT_REPO_ROOT
A=$1; B=$2; N=${3:-2}; SH=${4:-qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st}
O=$R/gpurun_out/r4ab
mkdir -p $O
for r in $(seq 1 $N); do
  for lib in $A $B; do
    tag=$(basename $lib .so)
    VTD_LIB_PATH=$R/$lib timeout -k 10 150 python tools/gemm_bench.py --shapes $SH --reps 20 > $O/gemm_${tag}_$r.jsonl 2>&1 || { tail -5 $O/gemm_${tag}_$r.jsonl; exit 1; }
    echo "$tag r$r gemm: $(python3 -c "import json,sys; print(' '.join(f\"{j['shape']}={j['us']}\" for j in map(json.loads, open('$O/gemm_${tag}_$r.jsonl'))))")"
    VTD_LIB_PATH=$R/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/bench_${tag}_$r.log 2>&1 || { tail -5 $O/bench_${tag}_$r.log; exit 1; }
    echo "$tag r$r bench: $(tail -1 $O/bench_${tag}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
