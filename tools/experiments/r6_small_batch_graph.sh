# small-batch latency: eager forward vs one HIP-graph replay per step (bench.py --graph 1), bf16x3 / bf16
set -o pipefail
for dt in bf16x3 bf16; do
  for b in 1 8 32; do
    for g in 0 1; do
      timeout -k 10 300 python bench.py --dtype $dt --batch $b --graph $g --steps 50 --warmup 10 --no-cpu-baseline --no-parity-mode 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$dt b=$b graph=$g', d['value'], 'img/s', d['ms_per_step'], 'ms')" || exit 1
    done
  done
done
