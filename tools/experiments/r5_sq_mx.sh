#!/bin/bash
# SQ counters of the MX-fp8 GEMM (C5 shapes + sq8192) next to the bf16 pp2 mlp2: where the
# MX K loop loses against the bf16 one.  Separate --pmc passes; mean per launch.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sqmx; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_COUNT"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P3="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
n=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/mx$n -o p --output-format csv -- python3 $R/tools/gemm_bench_mx.py --shapes qkv,mlp1,mlp2,sq8192 --variants 1 --reps 4 > $O/mx$n.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $P -d $O/bf$n -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes mlp2 --reps 4 > $O/bf$n.log 2>&1 || exit 1
  n=$((n+1))
done
cd $R
for n in 1 2 3; do python3 tools/pmc_summary.py $O/mx$n gemm_mx8 > $O/mx$n.txt; python3 tools/pmc_summary.py $O/bf$n pp2 > $O/bf$n.txt; done
cat $O/mx1.txt $O/mx2.txt $O/mx3.txt $O/bf1.txt $O/bf2.txt $O/bf3.txt
grep -h '"us"' $O/mx1.log $O/bf1.log || true
find $O -name '*counter_collection.csv' -delete
