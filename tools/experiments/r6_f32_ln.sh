# f32 parity mode LayerNorm pass: 16-column kernel vs the 4-column kernel (VTD_LN16_F32=0)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  VTD_LN16_F32=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6f32ln/prof$v -o p --output-format csv -- python3 $R/bench.py --dtype f32 --steps 3 --warmup 1 --no-cpu-baseline --no-parity-mode --streams 1 > /dev/null 2>&1 || exit 1
  f=$(find $R/gpurun_out/r6f32ln/prof$v -name '*kernel_stats.csv' | head -1)
  echo "VTD_LN16_F32=$v"; grep -i layernorm $f | cut -c1-200
  find $R/gpurun_out/r6f32ln -name '*kernel_trace.csv' -delete
done
cd $R
for v in 1 0 1 0; do
  VTD_LN16_F32=$v timeout -k 10 300 python bench.py --dtype f32 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('f32 ln16=$v', d['value'], d['ms_per_step'])" || exit 1
done
