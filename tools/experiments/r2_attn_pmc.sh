# attention at C2 alone: timing (MALL-warm and flushed) for variants 3 / 2, then PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in 3 2; do
  VTD_ATTN_VARIANT=$v timeout -k 10 120 python3 tools/attn_bench.py >> gpurun_out/r2_attn_micro.jsonl 2>/dev/null || exit 1
  VTD_ATTN_VARIANT=$v timeout -k 10 120 python3 tools/attn_bench.py --flush >> gpurun_out/r2_attn_micro.jsonl 2>/dev/null || exit 1
done
cat gpurun_out/r2_attn_micro.jsonl
cd /tmp && export TMPDIR=/tmp
export VTD_ATTN_VARIANT=3
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/attn_pmc0 -o p --output-format csv -- python3 $R/tools/attn_bench.py --reps 3 --flush > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/attn_pmc0w -o p --output-format csv -- python3 $R/tools/attn_bench.py --reps 3 --flush > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA -d $R/gpurun_out/attn_pmc1 -o p --output-format csv -- python3 $R/tools/attn_bench.py --reps 3 > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $R/gpurun_out/attn_pmc2 -o p --output-format csv -- python3 $R/tools/attn_bench.py --reps 3 > /dev/null 2>&1 || exit 1
echo ok
