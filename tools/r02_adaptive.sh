set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_adaptive.py tests/test_gpu_codec.py -k "adaptive" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02b_adaptive.log 2>&1; rc=$?
tail -30 gpurun_out/r02b_adaptive.log; exit $rc
