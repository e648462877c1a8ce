set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -k "1gib or randk" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r02k.log 2>&1; rc=$?; tail -12 gpurun_out/r02k.log; exit $rc
