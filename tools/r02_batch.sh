set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/batch_tests.log 2>&1; rc=$?; tail -12 gpurun_out/batch_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/batch_probe.py > gpurun_out/batch_probe.txt 2>&1; rc=$?; cat gpurun_out/batch_probe.txt; exit $rc
