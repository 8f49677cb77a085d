# persistent attention diagnostics: full / no-DMA / no-compute vs the per-pair kernel (C2 shape)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/ps_tests.log 2>&1 || { tail -30 gpurun_out/ps_tests.log; exit 1; }
tail -1 gpurun_out/ps_tests.log
rm -f gpurun_out/ps_micro.jsonl
for r in 1 2; do for v in "2 0" "4 0" "4 1" "4 2" "4 3"; do set -- $v
  VTD_ATTN_VARIANT=$1 VTD_ATTN_DIAG=$2 timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/ps_one.json 2>/dev/null || exit 1
  echo "{\"diag\": $2, \"r\": $(cat gpurun_out/ps_one.json)}" >> gpurun_out/ps_micro.jsonl
done; done
cat gpurun_out/ps_micro.jsonl
