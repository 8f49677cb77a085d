# PMC pass over the JPEG decode kernels (instruction mix and waits)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $R/gpurun_out/jpeg_pmc -o p --output-format csv -- python3 $R/tools/jpeg_bench.py --reps 1 > /dev/null 2>&1 || exit 1
echo ok
