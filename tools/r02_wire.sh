# packed-wire fold: GPU tests, then the bench's config4 leg (extras on, no CPU baseline)
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-wire}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_aggregation.py -k "wire or config3 or rccl" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -15 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --skip-cpu > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['extra']['config4_codec_plus_rccl_reduce_25M']))"
