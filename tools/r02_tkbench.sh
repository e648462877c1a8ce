# top-k / stacked GPU tests, the phase stamps of diag/lib_st.so, then the driver-shaped headline bench line
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-tk}
bash tools/r02_topkcheck.sh st || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --skip-extra --skip-cpu > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
