#!/bin/bash
# Kernel timeline (rocprofv3 --kernel-trace) of the headline step: durations and gaps of the last steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --skip-extra --skip-cpu > gpurun_out/tl.log 2>&1 || { tail gpurun_out/tl.log; exit 1; }
python3 tools/timeline.py $(find gpurun_out/tl -name "*kernel_trace.csv" | head -1) ${1:-16} | tee gpurun_out/timeline.txt
