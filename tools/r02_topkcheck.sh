# top-k / stacked GPU tests, then the phase stamps of diag/lib_st.so
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_torch_ops.py tests/test_gpu_aggregation.py -k "topk or stacked or tiles or sparse or config3 or fold or host" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/topkcheck.log 2>&1; rc=$?; tail -3 gpurun_out/topkcheck.log; [ $rc -ne 0 ] && exit $rc
bash tools/r02_variants.sh ${@:-st}
