# HIP runtime knobs A/B on the headline forward: kernel arguments in device memory.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c14
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/b_${v}_$r.log 2>&1 || { tail -5 $O/b_${v}_$r.log; exit 1; }
    echo "dev_kernarg=$v r$r $(tail -1 $O/b_${v}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
