# stamps of the 1 GiB encode for each diag/lib_*.so variant named on the command line
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  FLC_LIB=$PWD/diag/lib_$v.so ITERS=10 timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_$v.log 2>&1 || exit $?
  grep -E "^keys|^sample-sel" gpurun_out/stamps_$v.log | tail -2
  grep -E "^blocks|^kernel end" gpurun_out/stamps_$v.log
done
