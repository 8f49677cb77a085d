# Finalize grid-stride knob (test + forward A/B) and the pp2 realtime-stamp occupancy summary.
#   gpurun --timeout 900 -- bash tools/r4_check5.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c5
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "statout_and_finalize" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for rnd in 1 2; do
  for fw in 0 8 32; do
    VTD_FIN_WGS=$fw timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/b_$fw.log 2>&1 || { tail -20 $O/b_$fw.log; exit 1; }
    echo "fw=$fw $(tail -1 $O/b_$fw.log | cut -c1-120)"
  done
done
VTD_LIB_PATH=$R/vision_transformer_detector_amd/libvtd_diag.so VTD_PP2_DG=16 timeout -k 10 120 python tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st --reps 10 > $O/stamps.jsonl 2>&1 || { tail -20 $O/stamps.jsonl; exit 1; }
cat $O/stamps.jsonl
