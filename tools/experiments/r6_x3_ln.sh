# bf16x3 LayerNorm pass: 16-column kernel vs the 4-column kernel (VTD_LN16_X3=0), one-stream stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6x3ln
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  VTD_LN16_X3=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$v -o p --output-format csv -- python3 $R/bench.py --dtype bf16x3 --steps 5 --warmup 2 --no-cpu-baseline --no-parity-mode --streams 1 > $O/prof$v.log 2>&1 || { tail -20 $O/prof$v.log; exit 1; }
  f=$(find $O/prof$v -name '*kernel_stats.csv' | head -1)
  echo "VTD_LN16_X3=$v"; grep -i layernorm $f | cut -c1-200
  find $O -name '*kernel_trace.csv' -delete
done
cd $R
for v in 1 0 1 0; do
  VTD_LN16_X3=$v timeout -k 10 300 python bench.py --dtype bf16x3 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ln16=$v', d['value'], d['ms_per_step'])" || exit 1
done
