set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "accumulator_layouts or statout" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_diag.so VTD_PP2_DG=16 timeout -k 10 200 python tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st,qkv_h,attn_out_h,mlp2_h --reps 10 > $O/stamps.jsonl 2>&1 || { tail -20 $O/stamps.jsonl; exit 1; }
grep -o '"shape": "[a-z0-9_]*", "us": [0-9.]*\|"stamp_cycles": {[^}]*}' $O/stamps.jsonl
for r in 1 2; do for v in -1 1; do
  VTD_GEMM_TR=$v timeout -k 10 150 python tools/gemm_bench.py --shapes qkv_ln,attn_out_st --reps 20 > $O/tr_$v.jsonl 2>&1 || exit 1
  echo "TR=$v r$r: $(grep -o '"shape": "[a-z0-9_]*", "us": [0-9.]*' $O/tr_$v.jsonl | tr '\n' ' ')"
  VTD_GEMM_TR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/bench_tr_$v.log 2>&1 || exit 1
  echo "TR=$v r$r bench: $(tail -1 $O/bench_tr_$v.log | grep -o '"value": [0-9.]*')"
done; done
