set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_small
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS --kernel-trace -d gpurun_out/pmc_small/sq -o run --output-format csv -- python3 tools/small_configs.py > gpurun_out/pmc_small/sq.log 2>&1; rc=$?
echo "pmc rc=$rc"; exit $rc
