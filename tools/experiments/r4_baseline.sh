# Round-4 baseline on the GPU box: headline bench, per-shape GEMM timings (+ vendor library),
# per-shape PMC passes (FETCH_SIZE / WRITE_SIZE / TCC hit) of tools/gemm_bench.py, and the
# pp2 epilogue ablation of the diagnostic library (VTD_PP2_DG, wrong outputs).
#   gpurun --timeout 900 -- bash tools/r4_baseline.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
SH=qkv,qkv_ln,attn_out,attn_out_st,mlp1,mlp1_ln,mlp2,mlp3,mlp3_st,head1,head2,sq8192,mlp1_noact,mlp2_noact,qkv_h,attn_out_h,mlp1_h,mlp2_h,mlp3_h
VTD_GEMM_REF_LIB=1 timeout -k 10 240 python tools/gemm_bench.py --shapes $SH > $O/gemm.jsonl 2>&1 || { tail -20 $O/gemm.jsonl; exit 1; }
cat $O/gemm.jsonl
if [ -f vision_transformer_detector_amd/libvtd_diag.so ]; then
  for dg in 0 1 2 4 8; do
    VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_diag.so VTD_PP2_DG=$dg timeout -k 10 120 python tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st --reps 20 | sed "s/^/dg=$dg /" >> $O/ablation.jsonl || exit 1
  done
  cat $O/ablation.jsonl
fi
cd /tmp && export TMPDIR=/tmp
PS=qkv,attn_out,mlp1,mlp2,mlp3,head1,head2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pw.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pt -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $PS --reps 5 > $O/pt.log 2>&1 || exit 1
python3 $R/tools/pmc_per_shape.py $O/pf $O/pw $O/pt $O/traffic_per_shape.json
echo done
