set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_codec.py -k "delta or stacked" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02o_delta.log 2>&1; rc=$?; tail -25 gpurun_out/r02o_delta.log; exit $rc
