# PMC passes over the isolated GEMM shapes (tools/gemm_bench.py): where the pp2 main loop
# and epilogue spend wave cycles.  One pass per counter group (gfx950 slot limits).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/r2_pmc_list.txt 2>&1 || true
timeout -k 10 200 python3 $R/tools/gemm_bench.py --reps 10 --shapes mlp1,mlp1_noact,mlp2,mlp2_noact,qkv,attn_out,mlp3,sq8192 > $R/gpurun_out/r2_gemm_diag.jsonl 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC -d $R/gpurun_out/r2_pmc1 -o p --output-format csv -- python3 $R/tools/gemm_bench.py --reps 2 --shapes mlp1,mlp2,qkv,sq8192 > $R/gpurun_out/r2_pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE -d $R/gpurun_out/r2_pmc2 -o p --output-format csv -- python3 $R/tools/gemm_bench.py --reps 2 --shapes mlp1,mlp2,qkv,sq8192 > $R/gpurun_out/r2_pmc2.log 2>&1 || exit 1
echo ok
