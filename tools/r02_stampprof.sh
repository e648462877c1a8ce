set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/prof && export TMPDIR=/tmp
export FLC_LIB=$PWD/diag/lib_st.so
ITERS=6 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stp -o run --output-format csv -- python3 tools/stamps.py > gpurun_out/stp.log 2>&1 || exit $?
grep -E "^sample-sel" gpurun_out/stp.log | tail -3
f=$(find gpurun_out/prof/stp -name "*kernel_stats.csv" | head -1); cut -d, -f1-7 $f | cut -c1-200 | head -5
