#!/bin/bash
# Round-6 evidence on the GPU box (gpurun --timeout 1500 -- bash tools/r6_final.sh <tag>):
# full -m gpu suite, the headline bench line, the other BASELINE configs, per-mode accuracy,
# rocprofv3 kernel-trace stats (one stream and default), PMC FETCH / WRITE passes for the
# headline's `traffic`, per-shape GEMM traffic (incl. head2).  Outputs in gpurun_out/<tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r6f}
O=$R/gpurun_out/$T
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
for cfg in "c2_b64_bf16:--batch 64" "c3_b32_bf16:--preset vit_b16_640 --batch 32" \
           "c5_b128_bf16:--preset vit_l16_384 --batch 128 --dtype bf16 --steps 10 --warmup 3" \
           "c5_b128_fp8:--preset vit_l16_384 --batch 128 --dtype fp8 --steps 10 --warmup 3" \
           "c2_b256_f32:--dtype f32 --steps 10 --warmup 3" \
           "c2_b256_bf16x3:--dtype bf16x3 --steps 10 --warmup 3" \
           "c3_b32_bf16x3:--preset vit_b16_640 --batch 32 --dtype bf16x3 --steps 10 --warmup 3"; do
  lab=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-mode $args > $O/bench_$lab.log 2>&1 || { tail -20 $O/bench_$lab.log; exit 1; }
  echo "$lab $(tail -1 $O/bench_$lab.log | grep -o '"value": [0-9.]*\|"mfma_util_attn_mlp": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 200 python tools/accuracy_report.py --out $O/accuracy.json > $O/accuracy.log 2>&1 || { tail -20 $O/accuracy.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode --streams 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof2 -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity-mode --streams 1 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity-mode --streams 1 > $O/pmc_write.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/shape_fetch -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st,head2 --reps 5 > $O/shape_fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/shape_write -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st,head2 --reps 5 > $O/shape_write.log 2>&1 || exit 1
cd $R
python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/gemm_traffic.json
python3 tools/pmc_per_shape.py $O/shape_fetch $O/shape_write $O/shape_fetch $O/gemm_traffic_per_shape.json > $O/per_shape.txt 2>&1 || true
# attention at C3 (the long-sequence streaming kernel): SQ passes for VALU per MFMA
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_COUNT"
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/attn_t -o t --output-format csv -- python3 $R/tools/attn_bench.py --N 1600 --B 32 --H 12 --reps 5 > $O/attn_t.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P1 -d $O/attn_p1 -o p --output-format csv -- python3 $R/tools/attn_bench.py --N 1600 --B 32 --H 12 --reps 5 > $O/attn_p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P2 -d $O/attn_p2 -o p --output-format csv -- python3 $R/tools/attn_bench.py --N 1600 --B 32 --H 12 --reps 5 > $O/attn_p2.log 2>&1 || exit 1
cd $R
python3 tools/attn_pmc_summary.py $O > $O/attn_pmc.txt 2>&1 || true
f=$(find $O/prof2 -name '*kernel_trace.csv' | head -1)
python3 tools/trace_forward2.py $f 8 2 > $O/trace_summary.txt 2>&1 || true
find $O -name '*kernel_trace.csv' -delete
find $O -name '*counter_collection.csv' -size +20M -delete
echo done
