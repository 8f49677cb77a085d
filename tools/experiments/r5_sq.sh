#!/bin/bash
# SQ counters (VALU / MFMA instruction counts, LDS) of the C2 B=256 encoder GEMM shapes:
# separate --pmc passes over tools/gemm_bench.py, summarised per (kernel, grid)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SH=qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_COUNT"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d $O/p1 -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $SH --reps 5 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P2 -d $O/p2 -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes $SH --reps 5 > $O/p2.log 2>&1 || exit 1
cd $R
python3 tools/pmc_summary.py $O/p1 pp2 > $O/p1.txt
python3 tools/pmc_summary.py $O/p2 pp2 > $O/p2.txt
cat $O/p1.txt $O/p2.txt
find $O -name '*counter_collection.csv' -delete
