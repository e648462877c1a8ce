#!/bin/bash
# rocprofv3 kernel-trace summary of one bench run (no PMC counters here; see tools/pmc.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-prof}
shift || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/$TAG -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof/$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
cat gpurun_out/${TAG}_kernel_stats.csv 2>/dev/null | head -30
exit $rc
