# TR-layout staged epilogue (libvtd_trs.so, -DVTD_TRS=1): tests through that library, then an
# interleaved A/B of default / trs / trs + VTD_GEMM_TR=1 (per-shape + forward), 2 rounds.
#   gpurun --timeout 1200 -- bash tools/r4_check8.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c8
mkdir -p $O
T=$R/vision_transformer_detector_amd/libvtd_trs.so
VTD_LIB_PATH=$T timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "accumulator_layouts or 256_tile_path or statout_and_finalize or layernorm_fold or tiles_per_workgroup" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
VTD_LIB_PATH=$T timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch_parity.py > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
SH=qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st
for r in 1 2; do
  for v in base trs trs_tr1; do
    case $v in
      base) L=$R/vision_transformer_detector_amd/libvtd.so; E="";;
      trs) L=$T; E="";;
      trs_tr1) L=$T; E="VTD_GEMM_TR=1";;
    esac
    env VTD_LIB_PATH=$L $E timeout -k 10 150 python tools/gemm_bench.py --shapes $SH --reps 20 > $O/gemm_${v}_$r.jsonl 2>&1 || { tail -5 $O/gemm_${v}_$r.jsonl; exit 1; }
    echo "$v r$r gemm: $(python3 -c "import json; print(' '.join(f\"{j['shape']}={j['us']}\" for j in map(json.loads, (l for l in open('$O/gemm_${v}_$r.jsonl') if l.startswith('{')))))")"
    env VTD_LIB_PATH=$L $E timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/bench_${v}_$r.log 2>&1 || { tail -5 $O/bench_${v}_$r.log; exit 1; }
    echo "$v r$r bench: $(tail -1 $O/bench_${v}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
