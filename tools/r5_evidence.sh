# Round-5 evidence pass on the GPU box (gpurun --timeout 1200 -- bash tools/r5_evidence.sh <tag>):
# full -m gpu suite, the headline bench line (interleaved with the previous build for an A/B when
# libvtd_prev.so is present), per-mode accuracy of the goldens, rocprofv3 kernel-trace stats of the
# bench command (one stream and default), the PMC FETCH / WRITE passes for `traffic`.
# Outputs in gpurun_out/<tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r5e}
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
P=$R/vision_transformer_detector_amd/libvtd_prev.so
if [ -f $P ]; then
  for r in 1 2; do
    VTD_LIB_PATH=$P timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 20 > $O/ab_prev_$r.log 2>&1 || { tail -5 $O/ab_prev_$r.log; exit 1; }
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 20 > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
    echo "r$r prev $(tail -1 $O/ab_prev_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/ab_new_$r.log | grep -o '"value": [0-9.]*')"
  done
fi
timeout -k 10 200 python tools/accuracy_report.py --out $O/accuracy.json > $O/accuracy.log 2>&1 || { tail -20 $O/accuracy.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode --streams 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof2 -o p --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity-mode --streams 1 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity-mode --streams 1 > $O/pmc_write.log 2>&1 || exit 1
python3 $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/gemm_traffic.json
echo done
