# rocprofv3 PMC passes (separate runs) over tools/gemm_bench.py shapes: SHAPES=qkv,mlp2 bash tools/pmc_passes.sh
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SH=${SHAPES:-sq8192,qkv,attn_out}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM_WR SQ_LDS_DATA_FIFO_FULL GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE"
for i in 1 2 3; do
  eval P=\$P$i
  timeout -s KILL 90 rocprofv3 --pmc $P -d $R/gpurun_out/pmc$i -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $SH --reps 5 > $R/gpurun_out/pmc$i.log 2>&1
done
