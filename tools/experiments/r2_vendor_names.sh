# Kernel names / resources of the vendor library's GEMMs on the forward shapes (timing reference)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2_vendor_prof -o p --output-format csv -- python3 $R/tools/gemm_bench.py --reps 3 --shapes sq8192,mlp3,mlp2_noact,qkv > $R/gpurun_out/r2_vendor_prof.log 2>&1 || exit 1
echo ok
