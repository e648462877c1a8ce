#!/bin/bash
# HBM traffic of the float64 top-k (tools/topk64_probe.py: 25 M float64, k = 1 %) from rocprofv3 PMC counters, one
# counter per pass with --kernel-trace only, then tools/traffic.py -> gpurun_out/traffic64.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc64
export TMPDIR=/tmp
TAG=${1:-pmc64}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc64/${TAG}_$C -o run --output-format csv \
    -- python3 tools/topk64_probe.py > gpurun_out/pmc64/${TAG}_$C.log 2>&1
  rc=$?
  echo "pmc $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/traffic.py gpurun_out/pmc64 $TAG > gpurun_out/traffic64.json && cat gpurun_out/traffic64.json
