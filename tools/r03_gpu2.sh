#!/bin/bash
# round-3: targeted GPU tests of the changed kernels (TESTS), the adaptive-random profile, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03b}
TESTS=${TESTS:-tests/test_gpu_adaptive.py tests/test_gpu_wire.py tests/test_gpu_batch.py tests/test_gpu_comm.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_targeted.log 2>&1; rc=$?; tail -15 gpurun_out/${TAG}_targeted.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_adaptive -o run --output-format csv \
    -- python3 tools/adaptive_probe.py > gpurun_out/${TAG}_adaptive.log 2>&1 && grep -v '^[EW]2' gpurun_out/${TAG}_adaptive.log &&
find gpurun_out/prof/${TAG}_adaptive -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_adaptive_kernel_stats.csv \; &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log; exit $rc
