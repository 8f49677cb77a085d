set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/c2
timeout -k 10 200 python tools/tail_bench.py > gpurun_out/c2/tail.log 2>&1 || { tail -20 gpurun_out/c2/tail.log; exit 1; }
cat gpurun_out/c2/tail.log | grep shape
for r in 1 2; do
VTD_GEMM_REF_LIB=1 timeout -k 10 200 python tools/gemm_bench.py --shapes attn_out_st,mlp3_st,qkv_ln,mlp1_ln,mlp2,head2,attn_out,mlp3 > gpurun_out/c2/vendor_$r.log 2>&1 || { tail -20 gpurun_out/c2/vendor_$r.log; exit 1; }
done
grep shape gpurun_out/c2/vendor_1.log
