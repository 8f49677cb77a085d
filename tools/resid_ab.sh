set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx8.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 python -u tools/accuracy_report.py --out gpurun_out/acc_bf16res.json > gpurun_out/acc1.log 2>&1 || { tail -20 gpurun_out/acc1.log; exit 1; }
VTD_RESID_F32=1 timeout -k 10 200 python -u tools/accuracy_report.py --out gpurun_out/acc_f32res.json > gpurun_out/acc2.log 2>&1 || { tail -20 gpurun_out/acc2.log; exit 1; }
cat gpurun_out/acc1.log gpurun_out/acc2.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b1.log 2>&1 || { tail -20 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log
VTD_RESID_F32=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b2.log 2>&1 || { tail -20 gpurun_out/b2.log; exit 1; }
tail -1 gpurun_out/b2.log
