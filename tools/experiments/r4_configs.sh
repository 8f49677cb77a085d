# The other BASELINE configs' bench lines at HEAD (gpurun -- bash tools/r4_configs.sh <tag>).
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r4cfg}
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
