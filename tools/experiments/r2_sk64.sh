# stream-K at C2 B=64 (49 row tiles: every layer's last round is partial), SK off / on
set -o pipefail
for m in 0 1 0 1; do
  VTD_GEMM_SK=$m timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --batch 64 --streams 1 --no-cpu-baseline > gpurun_out/sk64_$m.json 2>&1 || { tail -5 gpurun_out/sk64_$m.json; exit 1; }
  tail -1 gpurun_out/sk64_$m.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SK=$m', d['value'], d['roofline']['frac'], d['kernels']['gemm']['avg_us'])"
done
