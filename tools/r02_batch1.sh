set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
true
export FLC_LIB=$PWD/diag/libflcodec_stamps.so
ITERS=8 timeout -k 10 120 python tools/stamps.py 25000000 > gpurun_out/stamps25M.log 2>&1 || exit $?
ITERS=8 timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps1G.log 2>&1 || exit $?
tail -12 gpurun_out/stamps25M.log; tail -12 gpurun_out/stamps1G.log
