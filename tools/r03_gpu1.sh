#!/bin/bash
# round-3 pass: GPU tests, the adaptive-random profile, the driver-shaped bench line and the headline rocprof summary.
# Each GPU step has its own time limit and the steps are chained with && (nothing runs after a failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1 && tail -2 gpurun_out/${TAG}_gpu_tests.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_adaptive -o run --output-format csv \
    -- python3 tools/adaptive_probe.py > gpurun_out/${TAG}_adaptive.log 2>&1 && cat gpurun_out/${TAG}_adaptive.log | grep -v '^W' &&
find gpurun_out/prof/${TAG}_adaptive -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_adaptive_kernel_stats.csv \; &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 &&
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench_line.json &&
bash tools/profile.sh ${TAG}_headline --skip-extra --skip-cpu --steps 20
