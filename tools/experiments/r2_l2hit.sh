# L2 (TCC) hit rate of the isolated GEMM shapes (pp2 default)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/l2hit -o p --output-format csv -- python3 $R/tools/gemm_bench.py --reps 2 --shapes qkv,attn_out,mlp1,mlp2,mlp3,sq8192 > $R/gpurun_out/l2hit.log 2>&1 || exit 1
echo ok
