# C3 attention PMC (tools/attn_pmc_summary.py): the default kernel, and knob 4-wave (VTD_ATTN_VARIANT unset vs 2 with N>128 -> 8 wave; use env VTD_ATTN_FORCE4 ... )
set -o pipefail
R=$GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_COUNT"
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/attn_t -o t --output-format csv -- python3 $R/tools/attn_bench.py --N 1600 --B 32 --H 12 --reps 5 > $O/attn_t.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P1 -d $O/attn_p1 -o p --output-format csv -- python3 $R/tools/attn_bench.py --N 1600 --B 32 --H 12 --reps 5 > $O/attn_p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P2 -d $O/attn_p2 -o p --output-format csv -- python3 $R/tools/attn_bench.py --N 1600 --B 32 --H 12 --reps 5 > $O/attn_p2.log 2>&1 || exit 1
cd $R
python3 tools/attn_pmc_summary.py $O
