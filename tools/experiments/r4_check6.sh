# Tiles per pp2 workgroup (VTD_GEMM_TPW): bit-exact tests, per-shape timings, forward A/B.
#   gpurun --timeout 900 -- bash tools/r4_check6.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c6
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "tiles_per_workgroup or 256_tile_path or accumulator_layouts or statout_and_finalize" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for tpw in 1 2 3; do
  VTD_GEMM_TPW=$tpw timeout -k 10 120 python tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st --reps 20 | sed "s/^/tpw=$tpw /" >> $O/gemm.jsonl || exit 1
done
cut -c1-140 $O/gemm.jsonl
for rnd in 1 2; do
  for tpw in 1 2 3; do
    VTD_GEMM_TPW=$tpw timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/b_$tpw.log 2>&1 || { tail -20 $O/b_$tpw.log; exit 1; }
    echo "tpw=$tpw $(tail -1 $O/b_$tpw.log | cut -c90-130)"
  done
done
