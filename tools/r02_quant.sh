set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_torch_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02i_quant.log 2>&1; rc=$?
tail -3 gpurun_out/r02i_quant.log; [ $rc -ne 0 ] && exit $rc
bash tools/r02_small.sh r02i
