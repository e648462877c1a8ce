set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregation.py -k "config3 or dist_fold" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02c_config3.log 2>&1; rc=$?
tail -8 gpurun_out/r02c_config3.log; exit $rc
