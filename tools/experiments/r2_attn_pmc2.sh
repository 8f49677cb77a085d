# PMC pass over the attention micro-benchmark: per-pair kernel (2) vs persistent (4)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 2 4; do for d in 0 1; do
  VTD_ATTN_VARIANT=$v VTD_ATTN_DIAG=$d timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU -d $R/gpurun_out/apmc_${v}_$d -o p --output-format csv -- python3 $R/tools/attn_bench.py --reps 5 > $R/gpurun_out/apmc_${v}_$d.log 2>&1 || exit 1
done; done
echo ok
