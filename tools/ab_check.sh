# GPU-box A/B check of a runtime switch: kernel + model parity tests, the logit-error
# report and one bench line per arm.   gpurun -- bash tools/ab_check.sh VAR=value
set -o pipefail
AB="$1"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx8.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 python -u tools/accuracy_report.py --out gpurun_out/acc_a.json > gpurun_out/acc_a.log 2>&1 || { tail -20 gpurun_out/acc_a.log; exit 1; }
env $AB timeout -k 10 200 python -u tools/accuracy_report.py --out gpurun_out/acc_b.json > gpurun_out/acc_b.log 2>&1 || { tail -20 gpurun_out/acc_b.log; exit 1; }
grep -h bfloat16 gpurun_out/acc_a.log gpurun_out/acc_b.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_a.log 2>&1 || { tail -20 gpurun_out/b_a.log; exit 1; }
env $AB timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_b.log 2>&1 || { tail -20 gpurun_out/b_b.log; exit 1; }
python3 - <<'PY'
import json
for arm in "ab":
    d = json.loads(open(f"gpurun_out/b_{arm}.log").read().strip().splitlines()[-1])
    print(arm, d["value"], d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
