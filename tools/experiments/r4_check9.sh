# Experiments: several tiles per workgroup (VTD_GEMM_TPW) and the TR-layout staged epilogue
# (libvtd_trs.so): tests of the trs build, per-shape timings, interleaved forward A/B.
#   gpurun --timeout 1200 -- bash tools/r4_check9.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c9
mkdir -p $O
T=$R/vision_transformer_detector_amd/libvtd_trs.so
B=$R/vision_transformer_detector_amd/libvtd.so
VTD_LIB_PATH=$T timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_batch_parity.py -k "accumulator_layouts or 256_tile_path or statout_and_finalize or layernorm_fold or tiles_per_workgroup or batch" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
SH=qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st
cfg() {  # name -> lib + env
  case $1 in
    base) echo "$B";; tpw2) echo "$B VTD_GEMM_TPW=2";; tpw3) echo "$B VTD_GEMM_TPW=3";;
    trs) echo "$T";; trs_tr1) echo "$T VTD_GEMM_TR=1";;
  esac
}
for v in base tpw2 tpw3 trs trs_tr1; do
  set -- $(cfg $v); L=$1; shift
  env VTD_LIB_PATH=$L "$@" timeout -k 10 150 python tools/gemm_bench.py --shapes $SH --reps 20 > $O/gemm_$v.jsonl 2>&1 || { tail -5 $O/gemm_$v.jsonl; exit 1; }
  echo "$v gemm: $(python3 -c "import json; print(' '.join(f\"{j['shape']}={j['us']}\" for j in map(json.loads, (l for l in open('$O/gemm_$v.jsonl') if l.startswith('{')))))")"
done
for r in 1 2; do
  for v in base tpw2 trs trs_tr1; do
    set -- $(cfg $v); L=$1; shift
    env VTD_LIB_PATH=$L "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/bench_${v}_$r.log 2>&1 || { tail -5 $O/bench_${v}_$r.log; exit 1; }
    echo "$v r$r bench: $(tail -1 $O/bench_${v}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
