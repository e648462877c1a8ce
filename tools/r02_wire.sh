set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -k "host" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02f_wire.log 2>&1; rc=$?
tail -5 gpurun_out/r02f_wire.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r02f_bench.log 2>&1; rc=$?
tail -1 gpurun_out/r02f_bench.log; exit $rc
