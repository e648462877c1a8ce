# full GPU test suite + smoke; TAG names the logs
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -5 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_smoke.log; exit $rc
