# Round-4 check 2: skinny / f32-256 / stagger tests, forward A/Bs (stagger, f32 256-tile),
# a two-stream forward trace (head section), SQ counters of the GEMM shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py -k "reshape_scatter or skinny or f32_256 or stagger or two_stream or seeded_full_config" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for v in 0 1 2; do
  VTD_STAGGER=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/fwd_stagger_$v.log 2>&1 || { tail -5 $O/fwd_stagger_$v.log; exit 1; }
  echo "stagger $v round $r: $(tail -1 $O/fwd_stagger_$v.log | cut -c60-110)"
done; done
for r in 1 2; do for v in 1 0; do
  VTD_F32_PP2=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --dtype f32 > $O/fwd_f32_$v.log 2>&1 || { tail -5 $O/fwd_f32_$v.log; exit 1; }
  echo "f32 pp2=$v round $r: $(tail -1 $O/fwd_f32_$v.log | cut -c60-110) $(tail -1 $O/fwd_f32_$v.log | grep -o '"frac": [0-9.]*')"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_forward2.py $f 8 > $O/trace_summary.txt 2>&1 || true
head -45 $O/trace_summary.txt
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_COUNT"
for i in 1 2; do
  eval P=\$P$i
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/sq$i -o p --output-format csv -- python3 $R/tools/gemm_bench.py --shapes qkv_ln,attn_out_st,mlp1_ln,mlp2,mlp3_st --reps 5 > $O/sq$i.log 2>&1 || exit 1
done
echo done
